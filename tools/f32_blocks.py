#!/usr/bin/env python3
"""Where the f32 speed mode's regional bias sits (experiment tool): renders C2
in f32 (seed X) and f64 (seeds Y, Z), computes the 16x16-block z-scores of
tests/f32_stats.py and prints the worst blocks (block column / row, image row
0 = bottom) and a coarse text map of the z-scores.

    python tools/f32_blocks.py [--spp 500] [--tuning k=v,...]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402

import f32_stats  # noqa: E402
import ray_tracing_weekend_amd as rtw  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--spp", type=int, default=500)
    ap.add_argument("--tuning", default="")
    a = ap.parse_args()
    soa, b = rtw.scenes.simple_soa(0x5EED0001)
    cam = b.with_image_width(1200).with_image_height(800).with_samples_per_pixel(a.spp).with_max_depth(50).build()

    def render(prec, seed, tuning=""):
        with rtw.Renderer(precision=prec) as r:
            for kv in filter(None, tuning.split(",")):
                k, v = kv.split("=")
                r.set_tuning(k, int(v))
            r.set_scene(soa)
            return r.render(cam, seed) / a.spp
    f32 = render(rtw.RTW_F32, 11, a.tuning)
    ref = render(rtw.RTW_F64, 22)
    oth = render(rtw.RTW_F64, 33)
    s = f32_stats.compare(f32, ref, oth)
    # the block map (same arithmetic as compare)
    blk = 16
    ok = ~(np.isnan(f32).any(-1) | np.isnan(ref).any(-1) | np.isnan(oth).any(-1))
    d32 = np.where(ok[..., None], f32 - ref, 0.0).mean(-1)
    d64 = np.where(ok[..., None], oth - ref, 0.0).mean(-1)
    B = lambda x: f32_stats._blocks(x, blk)
    cnt = B(ok.astype(np.float64)).sum(axis=(1, 3))
    var64 = B(d64 ** 2).sum(axis=(1, 3)) / np.maximum(cnt, 1)
    mref = B(np.where(ok, ref.mean(-1), 0.0)).sum(axis=(1, 3)) / np.maximum(cnt, 1)
    noise = np.sqrt(np.maximum(var64, 1e-300) / np.maximum(cnt, 1) + (4e-6 * np.abs(mref)) ** 2)
    z = B(d32).sum(axis=(1, 3)) / np.maximum(cnt, 1) / noise
    z[(cnt < blk * blk // 2) | (var64 <= 0)] = 0.0
    order = np.argsort(-np.abs(z), axis=None)[:25]
    worst = []
    for idx in order:
        by, bx = np.unravel_index(idx, z.shape)
        worst.append({"bx": int(bx), "by": int(by), "z": round(float(z[by, bx]), 2),
                      "mean_f32": round(float(B(np.where(ok, f32.mean(-1), 0.0)).sum(axis=(1, 3))[by, bx] /
                                              max(cnt[by, bx], 1)), 5),
                      "mean_f64": round(float(mref[by, bx]), 5)})
    print(json.dumps({"stats": s, "worst": worst}), flush=True)
    chars = " .:-=+*#%@"
    for by in range(z.shape[0] - 1, -1, -1):          # top row first
        line = "".join(("+" if z[by, bx] > 0 else "-") if abs(z[by, bx]) >= 4 else
                       ("." if abs(z[by, bx]) >= 2 else " ") for bx in range(z.shape[1]))
        print(f"{by:3d} |{line}|")


if __name__ == "__main__":
    main()
