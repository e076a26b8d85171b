#!/usr/bin/env python3
"""Where f32 (hit64) paths part from f64 (experiment tool, CPU): reads a
tools/trace_paths.py npz (per traced pixel, 64 samples x 64 segments of
{object id, t, origin xyz, direction xyz}) and, for every sample, finds the
first segment whose closest hit is another object (t differs at the f32
level from the first segment on: hit64's camera ray is f32).  Each divergence is classified by the object the ray starts on
(the previous segment's hit) and its material, and by whether one precision
re-hits that object (an acne re-hit: the entry of a Metal trap, DESIGN.md
§2b) where the other does not.  Build the trace library with the reference
rejection sampler in hit64 so both precisions draw the same words through
Metal bounces:

    TRACE_VAR=build/variants/traceref TRACE_FLAGS=-DRTW_HIT64_REF_SPHERE=1 \\
        python tools/trace_paths.py build
    TRACE_VAR=build/variants/traceref python tools/trace_paths.py run --out X.npz --pixels ...
    python tools/trace_divergence.py X.npz
"""
import collections
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

MAT = {0: "lambertian", 1: "metal", 2: "dielectric"}


def main(path):
    import ray_tracing_weekend_amd as rtw
    soa, _ = rtw.scenes.simple_soa(0x5EED0001)
    n_pl = len(soa.plane_mat)
    mtype = np.asarray(soa.mat_type)
    smat = np.asarray(soa.sphere_mat)

    def material(obj):
        if obj < 0:
            return "none"
        if obj < n_pl:
            return "plane"
        return MAT.get(int(mtype[smat[obj - n_pl]]), "other")

    z = np.load(path)
    f64, f32 = z["f64"], z["f32"]          # [pixel, sample, segment, 8]
    counts = collections.Counter()
    first_seg = []
    n_samples = 0
    for p in range(f64.shape[0]):
        for s in range(f64.shape[1]):
            a, b = f64[p, s], f32[p, s]
            n_samples += 1
            for k in range(a.shape[0]):
                ida, idb = int(a[k, 0]), int(b[k, 0])
                if ida == -2 and idb == -2:
                    break
                if ida == idb:     # the discrete path (object sequence); t differs at f32 level
                    continue
                prev = int(a[k - 1, 0]) if k > 0 else -1
                kind = "camera" if k == 0 else material(prev)
                rehit64, rehit32 = k > 0 and ida == prev, k > 0 and idb == prev
                tag = "f64 re-hit only" if rehit64 and not rehit32 else (
                    "f32 re-hit only" if rehit32 and not rehit64 else "other")
                same_origin = bool(np.array_equal(a[k, 2:5], b[k, 2:5]))
                counts[(kind, tag, "same origin" if same_origin else "origin differs")] += 1
                first_seg.append(k)
                break
    rows = [{"from": k[0], "event": k[1], "origin": k[2], "samples": v} for k, v in counts.most_common()]
    print(json.dumps({"samples": n_samples, "diverged": int(sum(counts.values())),
                      "median_first_segment": float(np.median(first_seg)) if first_seg else None,
                      "divergences": rows}, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
