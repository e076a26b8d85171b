#!/usr/bin/env python3
"""Where NaN samples come from, f32 (hit64) vs f64 at the same seed
(experiment tool; the RTW_NANORIGIN build, rtw_probes.hpp): per world object,
the samples whose throughput turned NaN at a Lambertian bounce off it -- a
point inside a light sphere (Sphere::pdf_value's sqrt of a negative,
sphere.rs:101-111) -- and the segments' closest hits per object (where the
f32 paths' extra segments go), f64 at a second seed as the noise floor.
Object ids: planes first, then spheres; -1: miss.

    python tools/nan_origins.py build
    python tools/nan_origins.py run [--spp 100] [--seed 5] [--tuning k=v,...]
"""
import argparse
import ctypes as C
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
VAR = os.environ.get("NAN_VAR", os.path.join(ROOT, "build", "variants", "nan"))
EXTRA = os.environ.get("NAN_FLAGS", "").split()   # extra -D flags of an experiment build


def build():
    cs = os.path.join(ROOT, "ray_tracing_weekend_amd", "csrc")
    b = os.path.join(ROOT, "ray_tracing_weekend_amd", "build")
    os.makedirs(VAR, exist_ok=True)
    common = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "-fno-slp-vectorize", "--offload-arch=gfx950",
              f"-I{cs}", f"-I{ROOT}/include"] + EXTRA
    subprocess.run(common + ["-ffp-contract=on", "-DRTW_NANORIGIN=f32", "-c", f"{cs}/render_f32.hip", "-o",
                             f"{VAR}/render_f32.o"], check=True)
    subprocess.run(common + ["-ffp-contract=off", "-DRTW_NANORIGIN=f64", "-c", f"{cs}/render_f64.hip", "-o",
                             f"{VAR}/render_f64.o"], check=True)
    subprocess.run(common + ["-ffp-contract=off", "-c", f"{cs}/capi.cpp", "-o", f"{VAR}/capi.o"], check=True)
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o", f"{VAR}/librtw.so",
                    f"{VAR}/render_f32.o", f"{VAR}/render_f64.o", f"{b}/render_f64_lgrid.o", f"{VAR}/capi.o", f"{b}/rtw_host.o", f"{b}/bvh.o",
                    "-ldl"], check=True)
    for f in ("render_f32.o", "render_f64.o", "capi.o"):
        os.remove(os.path.join(VAR, f))
    print("built", f"{VAR}/librtw.so")


def run(a):
    os.environ["RTW_LIB_OVERRIDE"] = os.path.join(VAR, "librtw.so")
    sys.path.insert(0, ROOT)
    import numpy as np
    import ray_tracing_weekend_amd as rtw
    soa, b = rtw.scenes.simple_soa(0x5EED0001)
    cam = b.with_image_width(1200).with_image_height(800).with_samples_per_pixel(a.spp).with_max_depth(50).build()
    n_pl = len(soa.plane_mat)
    sph = np.asarray(soa.spheres).reshape(-1, 4)
    lights = np.asarray(soa.lights).reshape(-1, 4)
    mtype = np.asarray(soa.mat_type)
    smat = np.asarray(soa.sphere_mat)
    out = {"spp": a.spp, "seed": a.seed, "tuning": a.tuning}
    counts, hits, rehits = {}, {}, {}
    for name, prec, seed in (("f32", rtw.RTW_F32, a.seed), ("f64", rtw.RTW_F64, a.seed),
                             ("f64_other_seed", rtw.RTW_F64, a.seed + 1)):
        lib = name[:3]
        rd = getattr(rtw._lib, f"rtw_probe_nan_read_{lib}")
        rd.argtypes = [C.c_void_p, C.c_size_t, C.c_int]
        rh = getattr(rtw._lib, f"rtw_probe_hit_read_{lib}")
        rh.argtypes = [C.c_void_p, C.c_size_t, C.c_int]
        n = 1 + n_pl + len(sph)
        buf = (C.c_ulonglong * n)()
        hbuf = (C.c_ulonglong * n)()
        half = 1 << 15                                    # rtw_probes.hpp: kNanSlots / 2
        full = (C.c_ulonglong * (half + n))()
        with rtw.Renderer(precision=prec) as r:
            for kv in filter(None, a.tuning.split(",")):
                k, v = kv.split("=")
                r.set_tuning(k, int(v))
            r.set_scene(soa)
            rd(buf, n, 1)
            rh(full, half + n, 1)
            img = r.render(cam, seed)
            st = r.stats
            assert rd(buf, n, 1) >= 0 and rh(full, half + n, 1) >= 0
        hbuf = full[:n]
        h2buf = full[half:half + n]
        c = np.array(buf[1:], dtype=np.int64)
        counts[name] = c
        hits[name] = np.array(hbuf[:], dtype=np.int64)   # [0]: misses, [1 + id]: closest hits
        rehits[name] = np.array(h2buf[:], dtype=np.int64)[1:]   # [id]: hits of the object hit just before
        out[name] = {"nan_origin_samples": int(c.sum()), "nan_pixels": int(np.isnan(img).any(-1).sum()),
                     "segments_per_sample": round(st.segments / st.samples, 5),
                     "segments_hist": int(hits[name].sum()), "misses": int(hits[name][0]),
                     "rehits": int(rehits[name].sum())}
    # closest hits per object: where the f32 paths' extra segments land, with
    # the f64 two-seed difference as the noise floor
    def hit_rows(x, y):
        z = (x - y) / np.sqrt(np.maximum(x + y, 1))
        order = np.argsort(-np.abs(z))[:20]
        rows = []
        for k in order:
            obj = int(k) - 1
            rec = {"object": obj, "a": int(x[k]), "b": int(y[k]), "z": round(float(z[k]), 1)}
            if obj >= n_pl:
                s = sph[obj - n_pl]
                rec.update(center=[round(float(v), 3) for v in s[:3]], radius=float(s[3]),
                           material=int(mtype[smat[obj - n_pl]]))
            rows.append(rec)
        return rows, float(np.sqrt(np.mean(z * z)))
    out["hits_f32_vs_f64"], out["hits_z_rms_f32_vs_f64"] = hit_rows(hits["f32"], hits["f64"])
    out["hits_f64_vs_f64_other_seed"], out["hits_z_rms_f64_seeds"] = hit_rows(hits["f64_other_seed"], hits["f64"])
    # re-hits of the object the ray starts on, per object
    def rehit_rows(x, y):
        z = (x - y) / np.sqrt(np.maximum(x + y, 1))
        order = np.argsort(-np.abs(z))[:15]
        return [{"object": int(k), "a": int(x[k]), "b": int(y[k]), "z": round(float(z[k]), 1),
                 "material": int(mtype[smat[int(k) - n_pl]]) if k >= n_pl else -1} for k in order]
    out["rehits_f32_vs_f64"] = rehit_rows(rehits["f32"], rehits["f64"])
    out["rehits_f64_vs_f64_other_seed"] = rehit_rows(rehits["f64_other_seed"], rehits["f64"])
    # per-sphere comparison: the spheres with the most NaN origins in either mode
    f32, f64 = counts["f32"], counts["f64"]
    top = np.argsort(-(f32 + f64))[:25]
    rows = []
    for k in top:
        if f32[k] + f64[k] == 0:
            break
        rec = {"object": int(k), "f32": int(f32[k]), "f64": int(f64[k])}
        if k >= n_pl:
            s = sph[k - n_pl]
            d = np.linalg.norm(lights[:, :3] - s[:3], axis=1)
            inside = np.nonzero(d < np.abs(lights[:, 3]) + abs(s[3]))[0]
            rec.update(center=[round(float(v), 4) for v in s[:3]], radius=float(s[3]),
                       material=int(mtype[smat[k - n_pl]]), overlapping_lights=inside.tolist())
        rows.append(rec)
    out["top_objects"] = rows
    z = (f32.sum() - f64.sum()) / max(np.sqrt(f32.sum() + f64.sum()), 1.0)
    out["origin_diff_z"] = round(float(z), 2)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("cmd", choices=["build", "run"])
    ap.add_argument("--spp", type=int, default=100)
    ap.add_argument("--seed", type=int, default=5)
    ap.add_argument("--tuning", default="")
    a = ap.parse_args()
    build() if a.cmd == "build" else run(a)
