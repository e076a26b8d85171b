#!/usr/bin/env python3
"""Where a render kernel's wave cycles go, by part of the segment loop
(experiment tool; the RTW_CLOCK build of librtw.so, rtw_probes.hpp): every
wave charges its shader-clock cycles between probes to the part it just ran.
The shares are of wave-cycles (a wave waiting on memory or on a barrier is
charged to the part it waits in); the probes themselves cost a few percent.

    python tools/clock_profile.py build       # here (hipcc, CPU)
    python tools/clock_profile.py run [--precision f64|f32] [--config C2|C3|C5] [--spp N] [--tuning k=v,...]
"""
import argparse
import ctypes as C
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
VAR = os.path.join(ROOT, "build", "variants", "clock")
PARTS = {0: "item pool + sample start", 1: "planes", 2: "closest hit", 3: "hit record", 4: "Lambertian",
         5: "light pdf", 6: "specular (one pass)", 7: "Metal", 8: "Dielectric", 9: "sample end",
         10: "wave tail", 11: "cooperative grid walk (stash, unstash)", 12: "loop head",
         13: "grid walk: setup", 14: "grid walk: pieces", 15: "grid walk: owners' pdf sums",
         16: "grid walk: owners' merges"}
CONFIGS = {"C2": (11, 1200, 800, 500), "C3": (50, 1920, 1080, 1024), "C5": (500, 1920, 1080, 256)}


def build():
    cs = os.path.join(ROOT, "ray_tracing_weekend_amd", "csrc")
    b = os.path.join(ROOT, "ray_tracing_weekend_amd", "build")
    os.makedirs(VAR, exist_ok=True)
    common = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "-fno-slp-vectorize", "--offload-arch=gfx950",
              f"-I{cs}", f"-I{ROOT}/include"]
    subprocess.run(common + ["-ffp-contract=on", "-DRTW_CLOCK=f32", "-c", f"{cs}/render_f32.hip", "-o",
                             f"{VAR}/render_f32.o"], check=True)
    subprocess.run(common + ["-ffp-contract=off", "-DRTW_CLOCK=f64", "-c", f"{cs}/render_f64.hip", "-o",
                             f"{VAR}/render_f64.o"], check=True)
    # (the f64 light-grid kernels, render_f64_lgrid.hip, from the in-tree build: without
    # probes -- their C3 / C5 f64 clock profiles need the probes in that unit, whose
    # readers would clash with render_f64.hip's)
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o", f"{VAR}/librtw.so",
                    f"{VAR}/render_f32.o", f"{VAR}/render_f64.o", f"{b}/render_f64_lgrid.o", f"{b}/capi.o",
                    f"{b}/rtw_host.o", f"{b}/bvh.o",
                    "-ldl"], check=True)
    print("built", f"{VAR}/librtw.so")


def run(a):
    os.environ["RTW_LIB_OVERRIDE"] = os.path.join(VAR, "librtw.so")
    sys.path.insert(0, ROOT)
    import ray_tracing_weekend_amd as rtw
    rd = getattr(rtw._lib, f"rtw_probe_clock_read_{a.precision}")
    rd.argtypes = [C.c_void_p, C.c_int]
    buf = (C.c_ulonglong * 20)()
    n, w, h, spp = CONFIGS[a.config]
    soa, b = rtw.scenes.simple_soa(0x5EED0001, n)
    cam = b.with_image_width(w).with_image_height(h).with_samples_per_pixel(a.spp or spp).with_max_depth(50).build()
    prec = rtw.RTW_F64 if a.precision == "f64" else rtw.RTW_F32
    with rtw.Renderer(precision=prec) as r:
        for kv in filter(None, a.tuning.split(",")):
            k, v = kv.split("=")
            r.set_tuning(k, int(v))
        r.set_scene(soa)
        r.render(cam, 3)             # the first render counts tile costs (index order)
        rd(buf, 1)
        r.render(cam, 4)
        st = r.get_stats()
        ms = r.get_timings(1)[0][0]
        assert rd(buf, 1) == 0
    tot = sum(buf[k] for k in PARTS)
    out = {"config": a.config, "precision": a.precision, "tuning": a.tuning, "spp": a.spp or spp,
           "kernel_ms": round(ms, 3), "segments": st.segments, "parts": {}}
    for k, name in PARTS.items():
        if buf[k]:
            out["parts"][name] = {"share": round(buf[k] / tot, 4), "ms_equiv": round(buf[k] / tot * ms, 2)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("cmd", choices=["build", "run"])
    ap.add_argument("--precision", default="f64")
    ap.add_argument("--config", default="C2")
    ap.add_argument("--spp", type=int, default=0)
    ap.add_argument("--tuning", default="")
    a = ap.parse_args()
    build() if a.cmd == "build" else run(a)
