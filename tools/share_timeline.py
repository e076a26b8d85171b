#!/usr/bin/env python3
"""Per-wave timeline of one render launch (experiment tool; needs the
RTW_TIMELINE build of librtw.so): every wave's begin / end wall-clock tick
(100 MHz), task count and XCD.  Prints where the launch spends its time: the
spread of wave start and end times, the idle tail, per-XCD end times.

    python tools/share_timeline.py build [--precision f64] # here (hipcc cross-compiles)
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


def build(precision):
    cs = os.path.join(ROOT, "ray_tracing_weekend_amd", "csrc")
    b = os.path.join(ROOT, "ray_tracing_weekend_amd", "build")
    os.makedirs(VAR, exist_ok=True)
    # the timeline probes in ONE precision's kernels (they define the read-back symbol)
    contract = "off" if precision == "f64" else "on"
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "-fno-slp-vectorize",
                    "--offload-arch=gfx950", f"-I{cs}", f"-I{ROOT}/include", f"-ffp-contract={contract}",
                    "-DRTW_TIMELINE", "-c", f"{cs}/render_{precision}.hip", "-o", f"{VAR}/render_{precision}.o"],
                   check=True)
    other = "f32" if precision == "f64" else "f64"
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o", f"{VAR}/librtw.so",
                    f"{VAR}/render_{precision}.o", f"{b}/render_{other}.o", f"{b}/capi.o", f"{b}/rtw_host.o",
                    f"{b}/bvh.o"], check=True)
    print("built", f"{VAR}/librtw.so")


def run(a):
    os.environ["RTW_LIB_OVERRIDE"] = os.path.join(ROOT, "build", "variants", a.variant, "librtw.so") \
        if a.variant else os.path.join(VAR, "librtw.so")
    sys.path.insert(0, ROOT)
    import numpy as np
    import torch
    import ray_tracing_weekend_amd as rtw
    rd = rtw._lib.rtw_probe_timeline_read
    rd.argtypes = [C.POINTER(C.c_ulonglong), C.c_size_t, C.c_int]
    n_tl = (1 << 16) * 8
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
    prec = rtw.RTW_F64 if a.precision == "f64" else rtw.RTW_F32
    tdt = torch.float64 if prec == rtw.RTW_F64 else torch.float32
    r = rtw.Renderer(precision=prec)
    for kv in filter(None, a.tuning.split(",")):
        k, v = kv.split("=")
        r.set_tuning(k, int(v))
    r.set_scene(scene)
    out = torch.empty((rtw.tiles_for_rank(W, H, 0, 1) * 64 * 3,), dtype=tdt, device="cuda:0")
    nb = out.numel() * out.element_size()
    r.render_device(cam, 1, out.data_ptr(), nb)
    for n in (int(x) for x in a.ns.split(",")):
        for _ in range(2):       # the counting render of this split, then one in the cached task order
            r.render_device(cam, 7, out.data_ptr(), nb, rank=min(a.rank, n - 1), nranks=n)
        torch.cuda.synchronize()
        rd(buf_tl, n_tl, 1)
        r.render_device(cam, 7, out.data_ptr(), nb, rank=min(a.rank, n - 1), nranks=n)
        torch.cuda.synchronize()
        kern = r.get_timings(1)[0][0]
        rd(buf_tl, n_tl, 1)
        t = np.frombuffer(buf_tl, dtype=np.uint64).reshape(-1, 8).astype(np.int64)
        t = t[t[:, 1] > 0]
        last_task = t[:, 2] >> 32
        t[:, 2] &= 0xFFFFFFFF
        hw = t[:, 3] >> 32
        t[:, 3] &= 0xF
        segs, last_t, dry_t, dry_trips = t[:, 4], t[:, 5], t[:, 6], t[:, 7]
        t0 = t[:, 0].min()
        beg, end = (t[:, 0] - t0) / 100.0, (t[:, 1] - t0) / 100.0     # microseconds
        span = end.max()
        busy = (end - beg).sum()
        q = lambda x, p: float(np.percentile(x, p))
        xcc = {int(x): round(float(end[t[:, 3] == x].max()) / 1e3, 3) for x in np.unique(t[:, 3])}
        print(json.dumps({
            "precision": a.precision, "nranks": n, "rank": min(a.rank, n - 1), "segments": int(r.get_stats().segments), "tuning": a.tuning, "kernel_ms": round(kern, 3), "waves": int(len(t)),
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
            # the 10 last waves: when they took their last task (ms), their lane-segments per us over the
            # launch vs the median wave's, their wave slot in the SIMD (HW_ID bits 3:0) and SIMD (5:4)
            "last10_took_last_task_ms": [round(float(x - t0) / 1e5, 3) for x in last_t[np.argsort(end)[-10:]]],
            "last10_seg_rate_vs_median": [round(float(x), 3) for x in
                                          (segs / (end - beg) / np.median(segs / (end - beg)))[np.argsort(end)[-10:]]],
            "last10_wave_slot": [int(x & 0xF) for x in hw[np.argsort(end)[-10:]]],
            # when each of the 10 last waves found the task counter dry (ms), and its trips after that
            "last10_dry_ms": [round(float(x - t0) / 1e5, 3) if x else None for x in dry_t[np.argsort(end)[-10:]]],
            "last10_trips_after_dry": [int(x) for x in dry_trips[np.argsort(end)[-10:]]],
            "dry_ms_p1_p50_max": [round(float(np.percentile(dry_t[dry_t > 0] - t0, p)) / 1e5, 3) for p in (1, 50, 100)],
            "trips_after_dry_p50_p99_max": [int(np.percentile(dry_trips, p)) for p in (50, 99, 100)],
            "last10_simd": [int((x >> 4) & 3) for x in hw[np.argsort(end)[-10:]]],
            # per wave slot: mean lane-segments per us relative to the mean, and tasks taken
            "seg_rate_by_wave_slot": {int(s_): round(float((segs / (end - beg))[(hw & 0xF) == s_].mean() /
                                                          (segs / (end - beg)).mean()), 3)
                                      for s_ in np.unique(hw & 0xF)},
            "tasks_by_wave_slot": {int(s_): round(float(t[:, 2][(hw & 0xF) == s_].mean()), 1)
                                   for s_ in np.unique(hw & 0xF)},
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
    ap.add_argument("--precision", default="f64", choices=["f32", "f64"])
    ap.add_argument("--variant", default="", help="run: build/variants/NAME/librtw.so (tools/build_variant.py "
                                                  "NAME -DRTW_TIMELINE ...) instead of the timeline build")
    a = ap.parse_args()
    build(a.precision) if a.mode == "build" else run(a)
