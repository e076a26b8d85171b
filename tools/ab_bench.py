#!/usr/bin/env python3
"""A/B timing of prebuilt librtw.so variants the way bench.py times the
headline: one fresh Renderer per (variant, mode) in its own process, W warm-up
renders, then K renders of the C2 workload timed by the library's HIP events
around the render kernel (rtw_get_timings), device-resident output.

    python tools/ab_bench.py --variants old,new [--modes f32,plain,f64] [--rounds 2]
      (variant = build/variants/<name>/librtw.so; "tree" = the in-tree library)
    python tools/ab_bench.py --one MODE           (internal: one measurement)

Modes: f32 (hit64, the headline), plain (f32, hit64 = 0), f64 (parity mode);
append ":key=val,..." for tuning overrides (e.g. f32:bvh_kind=1).
"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
W, H, SPP, DEPTH = 1200, 800, 500, 50


def one(mode, steps, warmup, size):
    sys.path.insert(0, ROOT)
    import numpy as np
    import torch
    import ray_tracing_weekend_amd as rtw
    name, _, tun = mode.partition(":")
    tuning = dict(kv.split("=") for kv in filter(None, tun.split(",")))
    prec = rtw.RTW_F64 if name == "f64" else rtw.RTW_F32
    if name == "plain":
        tuning.setdefault("hit64", "0")
    w, h, spp = size
    scene, b = rtw.scenes.simple_soa(0x5EED0001)
    cam = b.with_image_width(w).with_image_height(h).with_samples_per_pixel(spp).with_max_depth(DEPTH).build()
    dev = torch.device("cuda:0")
    with rtw.Renderer(device=0, precision=prec) as r:
        for k, v in tuning.items():
            r.set_tuning(k, int(v))
        r.set_scene(scene)
        buf = torch.empty((rtw.tiles_for_rank(w, h, 0, 1) * 64 * 3,),
                          dtype=torch.float32 if prec == rtw.RTW_F32 else torch.float64, device=dev)
        for k in range(warmup + steps):
            r.render_device(cam, 1000 + k, buf.data_ptr(), buf.numel() * buf.element_size())
        torch.cuda.synchronize()
        ms, _ = r.get_timings(steps)
        st = r.get_stats()
        kern = r.last_kernel()
    print(json.dumps({"mode": mode, "kernel_ms": round(float(np.mean(ms)), 3),
                      "min_ms": round(float(np.min(ms)), 3), "kernel": kern,
                      "node_visits_per_segment": round(st.node_visits / max(st.segments, 1), 3),
                      "sphere_tests_per_segment": round(st.sphere_tests / max(st.segments, 1), 3)}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="tree")
    ap.add_argument("--modes", default="f32,plain,f64")
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--size", default=f"{W}x{H}x{SPP}")
    ap.add_argument("--one")
    a = ap.parse_args()
    size = tuple(int(x) for x in a.size.split("x"))
    if a.one:
        one(a.one, a.steps, a.warmup, size)
        return
    for rd in range(a.rounds):
        for v in a.variants.split(","):
            env = dict(os.environ)
            if v != "tree":
                env["RTW_LIB_OVERRIDE"] = os.path.join(ROOT, "build", "variants", v, "librtw.so")
            for m in a.modes.split(";") if ";" in a.modes else a.modes.split(","):
                out = subprocess.run([sys.executable, __file__, "--one", m, "--steps", str(a.steps), "--warmup",
                                      str(a.warmup), "--size", a.size], env=env, capture_output=True, text=True,
                                     timeout=600)
                line = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
                if out.returncode != 0 or not line:
                    print(json.dumps({"variant": v, "mode": m, "error": out.stderr[-500:]}), flush=True)
                    sys.exit(1)
                d = json.loads(line[-1])
                print(json.dumps({"round": rd, "variant": v, **d}), flush=True)


if __name__ == "__main__":
    main()
