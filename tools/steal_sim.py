#!/usr/bin/env python3
"""Ray batches of the C2 render as the persistent kernel's waves see them, for
the lockstep traversal simulator tools/steal_sim.cpp (experiment tool).

The oracle traces whole samples (rtwo_trace_path); a wave's item pool is
emulated as the kernel runs it: tasks of 64 x `glen` items (pixel, sample),
sample-major (lane k of a fresh task takes pixel k // glen, sample k % glen),
a lane whose path ends takes the next free item, the next task starts when
the pool is handed out.  Every wave iteration emits the 64 lanes' current
segments: {o xyz, d xyz, excluded sphere id (the one the ray starts on, the
kernel's hit64 exclusion) or -1, skip (the ray re-hits its own isolated
sphere: the kernel skips the traversal), active}.

    python tools/steal_sim.py OUT.bin [--tiles 12] [--glen 32]
"""
import argparse
import os
import struct
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import oracle as O  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--tiles", type=int, default=12)
    ap.add_argument("--glen", type=int, default=32)
    ap.add_argument("--seed", type=int, default=5)
    a = ap.parse_args()
    sc = O.scene_simple(0x5EED0001)
    cam = O.camera_build(**dict(O.simple_camera_kw(), image_width=1200, image_height=800,
                                samples_per_pixel=500, max_depth=50))
    rng = np.random.default_rng(a.seed)
    tiles = [(int(rng.integers(0, 150)), int(rng.integers(0, 100))) for _ in range(a.tiles)]
    n_sph = len(sc.sphere_mat)
    iso = np.ones(n_sph, bool)   # approximation: every sphere isolated (C2: nearly all are)

    def items():
        for (tx, ty) in tiles:
            for q in range(64 * a.glen):
                px, c = q // a.glen, q % a.glen
                i, j = tx * 8 + (px & 7), ty * 8 + (px >> 3)
                yield i, j, c

    it = items()

    def next_path():
        try:
            i, j, s = next(it)
        except StopIteration:
            return None
        _, path = O.trace_path(cam, sc, 99, i, j, s, accel=O.ACCEL_BVH_CACHED)
        return path

    lanes = [next_path() for _ in range(64)]
    pos = [0] * 64
    batches = []
    while any(p is not None for p in lanes):
        rows = []
        for k in range(64):
            p = lanes[k]
            if p is None:
                rows.append((0, 0, 0, 0, 0, 0, -1, 0, 0))
                continue
            seg = p[pos[k]]
            prev = int(p[pos[k] - 1][6]) - 1 if pos[k] > 0 else -1   # object ids: plane 0, spheres 1..
            cur = int(seg[6]) - 1
            excl = prev if prev >= 0 else -1
            skip = 1 if (excl >= 0 and cur == excl and iso[excl]) else 0
            rows.append((*seg[:6], excl, skip, 1))
        batches.append(rows)
        for k in range(64):
            if lanes[k] is None:
                continue
            pos[k] += 1
            if pos[k] >= len(lanes[k]):
                lanes[k] = next_path()
                pos[k] = 0
    with open(a.out, "wb") as f:
        sph = np.asarray(sc.spheres, np.float64).reshape(-1, 4)
        f.write(struct.pack("<II", len(sph), len(batches)))
        f.write(sph.tobytes())
        for rows in batches:
            for r in rows:
                f.write(struct.pack("<6diii", *r[:6], int(r[6]), int(r[7]), int(r[8])))
    print(f"{len(batches)} wave iterations, {sum(r[8] for b in batches for r in b)} rays, "
          f"{sum(r[7] for b in batches for r in b)} skipped")


if __name__ == "__main__":
    main()
