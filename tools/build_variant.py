#!/usr/bin/env python3
"""Build an experiment variant of librtw.so with extra preprocessor defines
(RTW_* switches of the kernels) into build/variants/NAME/librtw.so -- the
render units recompiled, the host objects taken from the in-tree build.  The
A/B and timeline tools load it with RTW_LIB_OVERRIDE (tools/ab_bench.py
--variants NAME, tools/share_timeline.py run --variant NAME).

    python tools/build_variant.py NAME [-DRTW_X=1 ...] [--only f64]
"""
import argparse
import os
import subprocess
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CS = os.path.join(ROOT, "ray_tracing_weekend_amd", "csrc")
OBJ = os.path.join(ROOT, "ray_tracing_weekend_amd", "build")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("name")
    ap.add_argument("--only", choices=["f32", "f64"], default=None,
                    help="recompile one precision's render unit; the other from the in-tree build")
    a, defines = ap.parse_known_args()      # the rest: -DNAME=VALUE ...
    a.defines = [d for d in defines if d.startswith("-D")]
    if len(a.defines) != len(defines):
        ap.error(f"only -D defines may follow: {defines}")
    var = os.path.join(ROOT, "build", "variants", a.name)
    os.makedirs(var, exist_ok=True)
    precs = [a.only] if a.only else ["f32", "f64"]
    if "f64" in precs:
        precs.append("f64_lgrid")   # the f64 light-grid kernels' unit (render_f64_lgrid.hip)

    def compile_one(prec):
        contract = "off" if prec.startswith("f64") else "on"
        subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "-fno-slp-vectorize",
                        "--offload-arch=gfx950", f"-I{CS}", f"-I{ROOT}/include", f"-ffp-contract={contract}",
                        *a.defines, "-c", f"{CS}/render_{prec}.hip", "-o", f"{var}/render_{prec}.o"], check=True)

    with ThreadPoolExecutor(3) as ex:
        list(ex.map(compile_one, precs))
    objs = [f"{var}/render_{p}.o" if p in precs else f"{OBJ}/render_{p}.o" for p in ("f32", "f64", "f64_lgrid")]
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o", f"{var}/librtw.so",
                    *objs, f"{OBJ}/capi.o", f"{OBJ}/rtw_host.o", f"{OBJ}/bvh.o", "-ldl"], check=True)
    print("built", f"{var}/librtw.so")


if __name__ == "__main__":
    main()
