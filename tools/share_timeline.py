#!/usr/bin/env python3
"""Per-wave timeline of one render launch (experiment tool; needs the
RTW_TIMELINE build of librtw.so): every wave's begin / end wall-clock tick
(100 MHz), task count and XCD.  Prints where the launch spends its time: the
spread of wave start and end times, the idle tail, per-XCD end times.

    python tools/share_timeline.py build                  # here (hipcc cross-compiles)
    python tools/share_timeline.py run [--ns 1,8] [--rank K] [--tuning k=v,...]
                                       [--config C5 --spp 64]   (a bench_configs scene)
"""
import argparse
import ctypes as C
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
VAR = os.path.join(ROOT, "build", "variants", "timeline")


def build():
    cs = os.path.join(ROOT, "ray_tracing_weekend_amd", "csrc")
    b = os.path.join(ROOT, "ray_tracing_weekend_amd", "build")
    os.makedirs(VAR, exist_ok=True)
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "-fno-slp-vectorize", "--offload-arch=gfx950",
                    f"-I{cs}", f"-I{ROOT}/include", "-ffp-contract=on", "-DRTW_TIMELINE", "-c",
                    f"{cs}/render_f32.hip", "-o", f"{VAR}/render_f32.o"], check=True)
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o", f"{VAR}/librtw.so",
                    f"{VAR}/render_f32.o", f"{b}/render_f64.o", f"{b}/capi.o", f"{b}/rtw_host.o", f"{b}/bvh.o"],
                   check=True)
    print("built", f"{VAR}/librtw.so")


def run(a):
    os.environ["RTW_LIB_OVERRIDE"] = os.path.join(VAR, "librtw.so")
    sys.path.insert(0, ROOT)
    import numpy as np
    import torch
    import ray_tracing_weekend_amd as rtw
    rd = rtw._lib.rtw_probe_timeline_read
    rd.argtypes = [C.POINTER(C.c_ulonglong), C.c_size_t, C.c_int]
    n_tl = 1 << 18
    buf_tl = (C.c_ulonglong * n_tl)()
    W, H, SPP = 1200, 800, 500
    if a.config:
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        from bench_configs import CONFIGS, SEED
        cfg = CONFIGS[a.config]
        W, H, SPP = cfg["w"], cfg["h"], a.spp or cfg["spp"]
        scene, b = rtw.scenes.simple_soa(SEED, cfg["n"])
    else:
        scene, b = rtw.scenes.simple_soa()
    cam = b.with_image_width(W).with_image_height(H).with_samples_per_pixel(SPP).with_max_depth(50).build()
    r = rtw.Renderer(precision=rtw.RTW_F32)
    for kv in filter(None, a.tuning.split(",")):
        k, v = kv.split("=")
        r.set_tuning(k, int(v))
    r.set_scene(scene)
    out = torch.empty((rtw.tiles_for_rank(W, H, 0, 1) * 64 * 3,), dtype=torch.float32, device="cuda:0")
    r.render_device(cam, 1, out.data_ptr(), out.numel() * 4)
    for n in (int(x) for x in a.ns.split(",")):
        rd(buf_tl, n_tl, 1)
        r.render_device(cam, 7, out.data_ptr(), out.numel() * 4, rank=min(a.rank, n - 1), nranks=n)
        torch.cuda.synchronize()
        kern = r.get_timings(1)[0][0]
        rd(buf_tl, n_tl, 1)
        t = np.frombuffer(buf_tl, dtype=np.uint64).reshape(-1, 4).astype(np.int64)
        t = t[t[:, 1] > 0]
        last_task = t[:, 2] >> 32
        t[:, 2] &= 0xFFFFFFFF
        t0 = t[:, 0].min()
        beg, end = (t[:, 0] - t0) / 100.0, (t[:, 1] - t0) / 100.0     # microseconds
        span = end.max()
        busy = (end - beg).sum()
        q = lambda x, p: float(np.percentile(x, p))
        xcc = {int(x): round(float(end[t[:, 3] == x].max()) / 1e3, 3) for x in np.unique(t[:, 3])}
        print(json.dumps({
            "nranks": n, "rank": min(a.rank, n - 1), "segments": int(r.get_stats().segments), "tuning": a.tuning, "kernel_ms": round(kern, 3), "waves": int(len(t)),
            "span_ms": round(span / 1e3, 3),
            "begin_us_p50_p99_max": [round(q(beg, 50), 1), round(q(beg, 99), 1), round(float(beg.max()), 1)],
            "end_ms_p1_p50_p90_p99_max": [round(q(end, p) / 1e3, 3) for p in (1, 50, 90, 99)] + [round(span / 1e3, 3)],
            "wave_occupancy": round(busy / (len(t) * span), 4),
            # fraction of the waves still running at 10 %, 20 %, ... of the span
            "alive_at_10pct_steps": [round(float(((beg <= f * span) & (end > f * span)).mean()), 3)
                                     for f in np.arange(0.1, 1.0, 0.1)],
            "tasks_per_wave_p1_p50_p99": [int(q(t[:, 2], p)) for p in (1, 50, 99)],
            "xcc_end_ms": xcc,
            "last_tasks_of_the_10_last_waves": [int(x) for x in last_task[np.argsort(end)[-10:]]],
            "n_tasks_hint": "tasks [0, n_tasks1) phase 1 tile-major, then phase 2"}), flush=True)
    r.close()


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=["build", "run"])
    ap.add_argument("--ns", default="1,8")
    ap.add_argument("--tuning", default="")
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--config", default="", help="C3 / C5: a tools/bench_configs.py scene")
    ap.add_argument("--spp", type=int, default=0)
    a = ap.parse_args()
    build() if a.mode == "build" else run(a)
