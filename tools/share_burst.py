#!/usr/bin/env python3
"""Rank-share render time, single launches vs a back-to-back burst (no host
sync in between): separates per-launch effects (clock ramp, launch gaps) from
the kernel's own efficiency.  One JSON line per (N, mode).

    python tools/share_burst.py [--ns 1,8] [--burst 10] [--tuning k=v,...]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import ray_tracing_weekend_amd as rtw  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ns", default="1,8")
    ap.add_argument("--burst", type=int, default=10)
    ap.add_argument("--tuning", default="")
    ap.add_argument("--depth", type=int, default=50)
    a = ap.parse_args()
    W, H, SPP = 1200, 800, 500
    scene, b = rtw.scenes.simple_soa()
    cam = b.with_image_width(W).with_image_height(H).with_samples_per_pixel(SPP).with_max_depth(a.depth).build()
    r = rtw.Renderer(precision=rtw.RTW_F32)
    for kv in filter(None, a.tuning.split(",")):
        k, v = kv.split("=")
        r.set_tuning(k, int(v))
    r.set_scene(scene)
    buf = torch.empty((rtw.tiles_for_rank(W, H, 0, 1) * 64 * 3,), dtype=torch.float32, device="cuda:0")
    stream = rtw.torch_stream(torch.cuda.current_device())
    r.render_device(cam, 1, buf.data_ptr(), buf.numel() * 4, stream=stream)
    torch.cuda.synchronize()
    for n in (int(x) for x in a.ns.split(",")):
        single = []
        for _ in range(3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            r.render_device(cam, 7, buf.data_ptr(), buf.numel() * 4, rank=0, nranks=n, stream=stream)
            torch.cuda.synchronize()
            single.append((time.perf_counter() - t0) * 1e3)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(a.burst):
            r.render_device(cam, 7 + k, buf.data_ptr(), buf.numel() * 4, rank=0, nranks=n, stream=stream)
        torch.cuda.synchronize()
        burst = (time.perf_counter() - t0) * 1e3 / a.burst
        kern = r.get_timings(a.burst)[0]
        print(json.dumps({"nranks": n, "single_ms": round(min(single), 2), "burst_ms": round(burst, 2),
                          "burst_kernel_ms": [round(x, 2) for x in kern], "tuning": a.tuning, "depth": a.depth}), flush=True)
    r.close()


if __name__ == "__main__":
    main()
