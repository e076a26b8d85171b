#!/usr/bin/env python3
"""Throughput of the other SURVEY.md §8 configurations on ONE GPU (bench.py
measures C2, the headline): C3 = scenes::simple generator over a 100 x 100
grid (10k spheres), 1920x1080, 1024 spp; C5 = 1000 x 1000 grid (1M spheres),
1920x1080, 256 spp (BASELINE quotes C5 on 8 GPUs; this is the per-GPU rate);
C4 = C2's scene at 3840x2160, 4096 spp (8 GPUs in BASELINE; --c4-rows renders
a band of it).  One JSON line per config.

    python tools/bench_configs.py [--configs C3,C5] [--spp-scale 1.0] [--precision f64]
      (RTW_LIB_OVERRIDE=build/variants/<name>/librtw.so times a variant)
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import ray_tracing_weekend_amd as rtw  # noqa: E402

SEED = 0x5EED0001
CONFIGS = {
    "C3": dict(n=50, w=1920, h=1080, spp=1024),
    "C4": dict(n=11, w=3840, h=2160, spp=4096),
    "C5": dict(n=500, w=1920, h=1080, spp=256),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="C3,C5")
    ap.add_argument("--spp-scale", type=float, default=1.0, help="scale spp (quick runs)")
    ap.add_argument("--steps", type=int, default=1)
    ap.add_argument("--tuning", default="")
    ap.add_argument("--precision", choices=["f32", "f64"], default="f32")
    a = ap.parse_args()
    for name in a.configs.split(","):
        cfg = CONFIGS[name]
        spp = max(1, int(cfg["spp"] * a.spp_scale))
        t0 = time.perf_counter()
        scene, b = rtw.scenes.simple_soa(SEED, cfg["n"])
        t_gen = time.perf_counter() - t0
        cam = b.with_image_width(cfg["w"]).with_image_height(cfg["h"]).with_samples_per_pixel(spp) \
               .with_max_depth(50).build()
        r = rtw.Renderer(precision=rtw.RTW_F64 if a.precision == "f64" else rtw.RTW_F32)
        for kv in filter(None, a.tuning.split(",")):
            k, v = kv.split("=")
            r.set_tuning(k, int(v))
        t0 = time.perf_counter()
        r.set_scene(scene)
        t_stage = time.perf_counter() - t0
        dt_out = torch.float64 if a.precision == "f64" else torch.float32
        buf = torch.empty((rtw.tiles_for_rank(cfg["w"], cfg["h"], 0, 1) * 64 * 3,), dtype=dt_out, device="cuda:0")
        nbytes = buf.numel() * buf.element_size()
        r.render_device(cam, 1, buf.data_ptr(), nbytes)      # warm-up
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(a.steps):
            r.render_device(cam, 2 + k, buf.data_ptr(), nbytes)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / a.steps
        st = r.get_stats()
        render_ms, _ = r.get_timings(a.steps)
        samples = cfg["w"] * cfg["h"] * spp
        print(json.dumps({
            "config": name, "precision": a.precision, "tuning": a.tuning, "lib": os.environ.get("RTW_LIB_OVERRIDE", "tree"), "spheres": len(scene.sphere_mat), "lights": len(scene.lights),
            "width": cfg["w"], "height": cfg["h"], "spp": spp, "max_depth": 50,
            "msamples_s": round(samples / dt / 1e6, 1), "ms_per_render": round(dt * 1e3, 2),
            "kernel_ms": round(sum(render_ms) / len(render_ms), 2),
            "kernel": int(st.kernel), "chunk": int(st.chunk),
            "segments_per_sample": round(st.segments / st.samples, 4),
            "node_visits_per_segment": round(st.node_visits / max(st.segments, 1), 3),
            "sphere_tests_per_segment": round(st.sphere_tests / max(st.segments, 1), 3),
            "scene_gen_s": round(t_gen, 2), "scene_stage_s": round(t_stage, 2),
            "finite_fraction": float(torch.isfinite(buf.view(-1, 3)).all(-1).float().mean()),
        }), flush=True)
        r.close()


if __name__ == "__main__":
    main()
