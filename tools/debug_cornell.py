#!/usr/bin/env python3
"""Debug: cornell_box f64 GPU vs oracle -- first depth where pixels differ."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np
import ray_tracing_weekend_amd as rtw
from oracle import oracle as O

soa, b = rtw.scenes.cornell_box_soa()
for depth in (1, 2, 3, 4, 6, 8, 12, 20):
    cam = b.copy().with_image_width(40).with_image_height(40).with_samples_per_pixel(4).with_max_depth(depth).build()
    with rtw.Renderer(precision=rtw.RTW_F64) as r:
        r.set_accel(rtw.RTW_ACCEL_BRUTE)
        r.set_chunk(1)
        r.set_scene(soa)
        g = r.render(cam, 71)
    ocam = O.Camera()
    for name, _ in O.Camera._fields_:
        setattr(ocam, name, getattr(cam.raw, name))
    ref, st = O.render(ocam, O.Scene(**soa.__dict__), 71, chunk=1, accel=O.ACCEL_BRUTE)
    diff = np.argwhere((np.nan_to_num(g, nan=-7) != np.nan_to_num(ref, nan=-7)).any(-1))
    print(f"depth {depth}: {len(diff)} differing pixels")
    for (j, i) in diff[:4]:
        print("   ", j, i, g[j, i], ref[j, i])
    if len(diff):
        j, i = diff[0]
        for s in range(4):
            c, _ = O.trace_sample(ocam, O.Scene(**soa.__dict__), 71, int(i), int(j), s)
            print("      oracle sample", s, c)
        break
