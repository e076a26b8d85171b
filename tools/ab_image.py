#!/usr/bin/env python3
"""Render a C2-scene frame (f32, default tuning) and save the sums as .npy --
run once per library (RTW_LIB_OVERRIDE) and compare the files to check that a
kernel change keeps the image bit for bit.

    python tools/ab_image.py OUT.npy [--w 300 --h 200 --spp 16]
    python tools/ab_image.py --compare A.npy B.npy
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out", nargs="?")
    ap.add_argument("--compare", nargs=2)
    ap.add_argument("--w", type=int, default=300)
    ap.add_argument("--h", type=int, default=200)
    ap.add_argument("--spp", type=int, default=16)
    ap.add_argument("--n", type=int, default=11)
    a = ap.parse_args()
    if a.compare:
        x, y = (np.load(f) for f in a.compare)
        same = (x == y) | (np.isnan(x) & np.isnan(y))
        print(f"bit-identical pixels: {same.all(-1).mean():.6f}")
        sys.exit(0 if same.all() else 1)
    import ray_tracing_weekend_amd as rtw
    scene, b = rtw.scenes.simple_soa(0x5EED0001, a.n)
    cam = b.with_image_width(a.w).with_image_height(a.h).with_samples_per_pixel(a.spp).with_max_depth(50).build()
    with rtw.Renderer(precision=rtw.RTW_F32) as r:
        r.set_scene(scene)
        img = r.render(cam, 7)
        print("kernel", r.stats.kernel)
    np.save(a.out, img)


if __name__ == "__main__":
    main()
