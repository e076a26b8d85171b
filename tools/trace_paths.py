#!/usr/bin/env python3
"""Trace the same samples in f64 and f32 and find where their paths part
(experiment tool; needs the RTW_TRACE build of librtw.so).

    python tools/trace_paths.py build                 # here (hipcc cross-compiles)
    python tools/trace_paths.py run --out X.npz [--pixels i,j;i,j...] [--tuning hit64=1]

Each traced pixel's first 64 samples record, per segment, the ray (origin,
direction) and the closest hit (object id, t) -- rtw_probes.hpp RTW_TRACE.
Both precisions draw the same RNG words, so a path is the same in both until
a decision flips; the npz holds the records of f64 and f32 for every pixel.
"""
import argparse
import ctypes as C
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
VAR = os.environ.get("TRACE_VAR", os.path.join(ROOT, "build", "variants", "trace"))
EXTRA = os.environ.get("TRACE_FLAGS", "").split()   # extra -D flags of an experiment build


def build():
    cs = os.path.join(ROOT, "ray_tracing_weekend_amd", "csrc")
    b = os.path.join(ROOT, "ray_tracing_weekend_amd", "build")
    os.makedirs(VAR, exist_ok=True)
    common = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "-fno-slp-vectorize", "--offload-arch=gfx950",
              f"-I{cs}", f"-I{ROOT}/include"] + EXTRA
    subprocess.run(common + ["-ffp-contract=on", "-DRTW_TRACE=f32", "-c", f"{cs}/render_f32.hip", "-o",
                             f"{VAR}/render_f32.o"], check=True)
    subprocess.run(common + ["-ffp-contract=off", "-DRTW_TRACE=f64", "-c", f"{cs}/render_f64.hip", "-o",
                             f"{VAR}/render_f64.o"], check=True)
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o", f"{VAR}/librtw.so",
                    f"{VAR}/render_f32.o", f"{VAR}/render_f64.o", f"{b}/render_f64_lgrid.o", f"{b}/capi.o", f"{b}/rtw_host.o", f"{b}/bvh.o"],
                   check=True)
    print("built", f"{VAR}/librtw.so")


def run(a):
    os.environ["RTW_LIB_OVERRIDE"] = os.path.join(VAR, "librtw.so")
    sys.path.insert(0, ROOT)
    import numpy as np
    import ray_tracing_weekend_amd as rtw
    lib = rtw._lib
    W, H, SPP = 1200, 800, 64
    soa, b = rtw.scenes.simple_soa(0x5EED0001)
    cam = b.with_image_width(W).with_image_height(H).with_samples_per_pixel(SPP).with_max_depth(50).build()
    pixels = [tuple(int(v) for v in p.split(",")) for p in a.pixels.split(";")]
    tuning = [(k, int(v)) for k, v in (kv.split("=") for kv in filter(None, a.tuning.split(",")))]
    out = {}
    n = 64 * 64 * 8
    buf = (C.c_double * n)()
    for prec, tag in ((rtw.RTW_F64, "f64"), (rtw.RTW_F32, "f32")):
        setf = getattr(lib, f"rtw_probe_trace_set_{tag}")
        setf.argtypes = [C.c_ulonglong]
        readf = getattr(lib, f"rtw_probe_trace_read_{tag}")
        readf.argtypes = [C.c_void_p, C.c_size_t]
        recs = []
        with rtw.Renderer(precision=prec) as r:
            if prec == rtw.RTW_F32:
                for k, v in tuning:
                    r.set_tuning(k, v)
            r.set_tuning("partial_max", 1 << 33)
            r.set_scene(soa)
            for (i, j) in pixels:
                assert setf(j * W + i) == 0
                r.render(cam, 5)
                assert readf(buf, n) == n
                recs.append(np.frombuffer(buf, np.float64).reshape(64, 64, 8).copy())
        out[tag] = np.stack(recs)
    np.savez_compressed(a.out, pixels=np.array(pixels), **out)
    f64, f32 = out["f64"], out["f32"]
    same_paths = ((f64[..., 0] == f32[..., 0]) | (f64[..., 0] == -2)).all(-1)
    print(f"pixels {len(pixels)}: samples with identical hit sequences {same_paths.mean():.3f}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=["build", "run"])
    ap.add_argument("--out", default="gpurun_out/trace.npz")
    ap.add_argument("--pixels", default=";".join(f"{i},{j}" for i in range(780, 900, 30) for j in (520, 560, 600, 640)))
    ap.add_argument("--tuning", default="")
    a = ap.parse_args()
    build() if a.mode == "build" else run(a)


if __name__ == "__main__":
    main()
