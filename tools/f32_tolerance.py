#!/usr/bin/env python3
"""f32 speed mode vs f64 parity mode at the headline configuration (C2:
1200x800, 500 spp, depth 50 on scenes::simple): the two-sample statistics of
tests/f32_stats.py (image-mean bias, variance ratio, regional block z, per-pixel
z, NaN fractions) and segments / Lambertian bounces per sample of both modes.
Prints one JSON line.  GPU; the f64 renders are the reference (bit-identical to
the oracle: tests/test_gpu_parity.py, bench.py's parity leg).

    python tools/f32_tolerance.py [--size 1200x800] [--spp 500] [--tuning k=v,...]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import ray_tracing_weekend_amd as rtw  # noqa: E402
import f32_stats  # noqa: E402


def render(soa, cam, seed, prec, tuning=()):
    with rtw.Renderer(device=0, precision=prec) as r:
        for k, v in tuning:
            r.set_tuning(k, v)
        r.set_scene(soa)
        img = r.render(cam, seed)
        st = r.stats
        return img / cam.samples_per_pixel, {"segments_per_sample": st.segments / st.samples,
                                             "lambertian_per_sample": st.lambertian / st.samples,
                                             "kernel_ms": round(st.kernel_ms, 2), "chunk": int(st.chunk)}


def measure(W=1200, H=800, spp=500, depth=50, seeds=(11, 22, 33), tuning=(), save=None):
    soa, b = rtw.scenes.simple_soa(0x5EED0001)
    cam = b.with_image_width(W).with_image_height(H).with_samples_per_pixel(spp).with_max_depth(depth).build()
    f32, s32 = render(soa, cam, seeds[0], rtw.RTW_F32, tuning)
    ref, s64 = render(soa, cam, seeds[1], rtw.RTW_F64)
    oth, _ = render(soa, cam, seeds[2], rtw.RTW_F64)
    out = f32_stats.compare(f32, ref, oth)
    if save:
        import numpy as np
        np.savez_compressed(save, f32=f32.astype(np.float32), ref=ref.astype(np.float32),
                            other=oth.astype(np.float32))
    out.update({"size": f"{W}x{H}", "spp": spp, "depth": depth, "seeds": list(seeds),
                "f32": s32, "f64": s64, "tuning": dict(tuning)})
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", default="1200x800")
    ap.add_argument("--spp", type=int, default=500)
    ap.add_argument("--tuning", default="")
    ap.add_argument("--save", default="", help="write the three mean images (npz, float32)")
    a = ap.parse_args()
    W, H = (int(x) for x in a.size.split("x"))
    tuning = tuple((k, int(v)) for k, v in (kv.split("=") for kv in filter(None, a.tuning.split(","))))
    print(json.dumps(measure(W, H, a.spp, tuning=tuning, save=a.save or None)), flush=True)


if __name__ == "__main__":
    main()
