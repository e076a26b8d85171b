#!/usr/bin/env python3
"""Regenerate the committed golden fixtures of tests/golden/ from the CPU
oracle (oracle/liboracle.so).  The Rust reference cannot run here (no cargo /
rustc) and its own tests hold no numeric fixtures, so these are
oracle outputs at fixed seeds: they pin the oracle against regressions and
give the GPU parity tests bit-level targets that need no CPU render.

    python tests/golden/make_golden.py
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import oracle as O  # noqa: E402

SCENE_SEED = 0x5EED0001
RENDER_SEED = 0xC0FFEE
# (name, camera overrides, chunk, window rows, window cols)
CASES = [
    # C1 geometry (BASELINE.json configs[0]): 400x225, 100 spp, depth 50 -- a
    # 32 x 8 window of it (the full C1 render takes minutes on the oracle)
    ("c1_window", dict(image_width=400, image_height=225, samples_per_pixel=100, max_depth=50),
     2, (104, 112, 1), (184, 216)),
    # a full small frame of the same scene, several chunks per pixel
    ("simple_48x27", dict(image_width=48, image_height=27, samples_per_pixel=16, max_depth=50),
     2, None, None),
]


def scene_fixture():
    sc = O.scene_simple(SCENE_SEED)
    return {k: np.asarray(getattr(sc, k)).tolist() for k in
            ("spheres", "sphere_mat", "planes", "plane_mat", "mat_type", "mat_params", "lights")}


def main():
    with open(os.path.join(HERE, "simple_scene_5EED0001.json"), "w") as f:
        json.dump({"seed": SCENE_SEED, "generator": "scenes::simple (scenes/src/lib.rs:155-233) "
                   "restated with xoshiro256++/splitmix64", **scene_fixture()}, f)
    sc = O.scene_simple(SCENE_SEED)
    arrays = {}
    for name, over, chunk, rows, cols in CASES:
        kw = dict(O.simple_camera_kw())
        kw.update(over)
        cam = O.camera_build(**kw)
        img, st = O.render(cam, sc, RENDER_SEED, chunk=chunk, accel=O.ACCEL_BVH_CACHED,
                           rows=rows, cols=cols)
        if rows is not None:
            img = img[rows[0]:rows[1], cols[0]:cols[1]]
        arrays[name] = img
        arrays[name + "_meta"] = np.array([chunk, st.samples, st.segments, st.lambertian,
                                           st.nan_samples], np.int64)
        print(name, img.shape, "segments/sample %.4f" % (st.segments / st.samples))
    np.savez_compressed(os.path.join(HERE, "golden_renders.npz"), **arrays)


if __name__ == "__main__":
    main()
