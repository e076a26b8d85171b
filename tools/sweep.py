#!/usr/bin/env python3
"""Tuning sweep on the GPU: C2 (1200x800x500spp, depth 50) render time for
scheduling / world-mode variants, interleaved rounds in one process."""
import argparse
import itertools
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import ray_tracing_weekend_amd as rtw  # noqa: E402


BUILD_KEYS = ("bvh_leaf", "light_leaf", "light_grid", "light_bvh_min")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--spp", type=int, default=500)
    ap.add_argument("--depth", type=int, default=50)
    ap.add_argument("--precision", default="f32")
    ap.add_argument("--grid", default="auto_chunk=4,8,16;target_tasks=65536,131072;lds=1,0")
    ap.add_argument("--accel", type=int, default=0)
    a = ap.parse_args()
    prec = rtw.RTW_F32 if a.precision == "f32" else rtw.RTW_F64
    scene, b = rtw.scenes.simple_soa()
    W, H = 1200, 800
    cam = b.with_image_width(W).with_image_height(H).with_samples_per_pixel(a.spp).with_max_depth(a.depth).build()
    keys, vals = [], []
    for part in a.grid.split(";"):
        k, v = part.split("=")
        keys.append(k)
        vals.append([int(x) for x in v.split(",")])
    combos = list(itertools.product(*vals))
    r = rtw.Renderer(precision=prec)
    r.set_accel(a.accel)
    r.set_scene(scene)
    buf = torch.zeros((H, W, 3), dtype=torch.float32 if prec == rtw.RTW_F32 else torch.float64,
                      device="cuda:0")
    res = {c: [] for c in combos}
    staged = {}
    for rd in range(a.rounds + 1):
        for c in combos:
            for k, v in zip(keys, c):
                r.set_tuning(k, v)
            # leaf sizes and the light grid are built at set_scene
            build = {k: v for k, v in zip(keys, c) if k in BUILD_KEYS}
            if build and staged.get("build") != build:
                r.set_scene(scene)
                staged["build"] = build
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            r.render_device(cam, 5 + rd, buf.data_ptr(), buf.numel() * buf.element_size())
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            if rd > 0:
                res[c].append(dt)
    st = r.get_stats()
    for c in combos:
        ms = min(res[c]) * 1e3
        print(json.dumps({"cfg": dict(zip(keys, c)), "ms": round(ms, 2),
                          "msamples_s": round(W * H * a.spp / (ms * 1e-3) / 1e6, 1)}), flush=True)
    print(json.dumps({"segments_per_sample": st.segments / max(st.samples, 1),
                      "lambertian_per_sample": st.lambertian / max(st.samples, 1),
                      "node_visits_per_segment": st.node_visits / max(st.segments, 1),
                      "sphere_tests_per_segment": st.sphere_tests / max(st.segments, 1)}))


if __name__ == "__main__":
    main()
