#!/usr/bin/env python3
"""Lane occupancy of the f32 render kernel by phase (experiment tool; needs the
RTW_PROF build of librtw.so): at each RTW_PROBE_LANES site the kernel counts
the wave passes and their active lanes (rtw_probes.hpp).

    python tools/lane_profile.py build        # here
    python tools/lane_profile.py run [--tuning k=v,...] [--spp 500]
"""
import argparse
import ctypes as C
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
VAR = os.path.join(ROOT, "build", "variants", "prof")
NAMES = {1: "bvh inner step", 2: "leaf tests", 3: "segment loop (wave)", 4: "segment (active lanes)",
         5: "own-sphere f64 test", 6: "closest-hit query", 7: "Metal", 8: "Dielectric", 9: "Lambertian",
         10: "next sample", 11: "grid walk: piece (f32 coop)", 12: "grid walk: light slot (f32 coop, 4 per cell)",
         13: "f64 walk: owner merge iteration", 14: "f64 walk: merged piece slot", 15: "f64 walk: dealt pdf pass"}
CONFIGS = {"C2": (11, 1200, 800, 500), "C3": (50, 1920, 1080, 1024), "C5": (500, 1920, 1080, 256)}


def build():
    cs = os.path.join(ROOT, "ray_tracing_weekend_amd", "csrc")
    b = os.path.join(ROOT, "ray_tracing_weekend_amd", "build")
    os.makedirs(VAR, exist_ok=True)
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "-fno-slp-vectorize", "--offload-arch=gfx950",
                    f"-I{cs}", f"-I{ROOT}/include", "-ffp-contract=on", "-DRTW_PROF=f32", "-c", f"{cs}/render_f32.hip",
                    "-o", f"{VAR}/render_f32.o"], check=True)
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "-fno-slp-vectorize", "--offload-arch=gfx950",
                    f"-I{cs}", f"-I{ROOT}/include", "-ffp-contract=off", "-DRTW_PROF=f64", "-c", f"{cs}/render_f64.hip",
                    "-o", f"{VAR}/render_f64.o"], check=True)
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o", f"{VAR}/librtw.so",
                    f"{VAR}/render_f32.o", f"{VAR}/render_f64.o", f"{b}/render_f64_lgrid.o", f"{b}/capi.o", f"{b}/rtw_host.o", f"{b}/bvh.o",
                    "-ldl"], check=True)
    print("built", f"{VAR}/librtw.so")


def run(a):
    os.environ["RTW_LIB_OVERRIDE"] = os.path.join(VAR, "librtw.so")
    sys.path.insert(0, ROOT)
    import ray_tracing_weekend_amd as rtw
    rd = getattr(rtw._lib, f"rtw_probe_lanes_read_{a.precision}")
    rd.argtypes = [C.c_void_p, C.c_int]
    buf = (C.c_ulonglong * 32)()
    n, w, h, _ = CONFIGS[a.config]
    soa, b = rtw.scenes.simple_soa(0x5EED0001, n)
    cam = b.with_image_width(w).with_image_height(h).with_samples_per_pixel(a.spp).with_max_depth(50).build()
    with rtw.Renderer(precision=rtw.RTW_F64 if a.precision == "f64" else rtw.RTW_F32) as r:
        for kv in filter(None, a.tuning.split(",")):
            k, v = kv.split("=")
            r.set_tuning(k, int(v))
        r.set_scene(soa)
        rd(buf, 1)
        r.render(cam, 3)
        st = r.get_stats()
        assert rd(buf, 1) == 0
    segs = st.segments
    out = {"config": a.config, "precision": a.precision, "tuning": a.tuning, "spp": a.spp, "segments": segs, "lambertian": st.lambertian, "phases": {}}
    for i, name in NAMES.items():
        lanes, passes = buf[2 * i], buf[2 * i + 1]
        if passes:
            out["phases"][name] = {"passes_per_64_segments": round(passes / segs * 64, 3),
                                   "lanes_per_pass": round(lanes / passes, 2),
                                   "lane_events_per_segment": round(lanes / segs, 3)}
    print(json.dumps(out), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=["build", "run"])
    ap.add_argument("--tuning", default="")
    ap.add_argument("--spp", type=int, default=500)
    ap.add_argument("--config", default="C2")
    ap.add_argument("--precision", default="f32")
    a = ap.parse_args()
    build() if a.mode == "build" else run(a)


if __name__ == "__main__":
    main()
