#!/usr/bin/env python3
"""Debug: C5-scene BVH vs brute force (f32 and f64) -- which pixels differ."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np
import ray_tracing_weekend_amd as rtw

soa, b = rtw.scenes.simple_soa(0x5EED0001, int(sys.argv[1]) if len(sys.argv) > 1 else 500)
cam = b.with_image_width(24).with_image_height(16).with_samples_per_pixel(2).with_max_depth(20).build()
for prec in (rtw.RTW_F32, rtw.RTW_F64):
    out = {}
    for accel in (rtw.RTW_ACCEL_BRUTE, rtw.RTW_ACCEL_BVH):
        for depth in (1, 20):
            c = b.copy().with_image_width(24).with_image_height(16).with_samples_per_pixel(2) \
                 .with_max_depth(depth).build()
            with rtw.Renderer(precision=prec) as r:
                r.set_tuning("light_bvh_min", 1 << 30)
                r.set_accel(accel)
                r.set_scene(soa)
                img = r.render(c, 43)
                out[(accel, depth)] = (np.nan_to_num(img, nan=-7.0), r.stats.segments, r.stats.kernel)
    for depth in (1, 20):
        a, bb = out[(rtw.RTW_ACCEL_BRUTE, depth)], out[(rtw.RTW_ACCEL_BVH, depth)]
        diff = np.argwhere((a[0] != bb[0]).any(-1))
        print(f"prec {prec} depth {depth}: kernels {a[2]}/{bb[2]} segs {a[1]}/{bb[1]} differing px {len(diff)}")
        for (j, i) in diff[:5]:
            print("   ", j, i, a[0][j, i], bb[0][j, i])
