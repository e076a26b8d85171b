import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import ray_tracing_weekend_amd as rtw
from oracle import oracle as O

def scene(plane=True, nested=True, invisible=True, inside_light=True, two_lights=True, metal=True):
    world = rtw.HittableList()
    if plane: world.add(rtw.Plane((0, -0.5, 0), (0, -1, 0), rtw.Lambertian((0.8, 0.8, 0.0))))
    world.add(rtw.Sphere((0, 0, -1.2), 0.5, rtw.Lambertian((0.1, 0.2, 0.5))))
    world.add(rtw.Sphere((-1, 0, -1), 0.5, rtw.Dialectric(1.5)))
    if nested: world.add(rtw.Sphere((-1, 0, -1), 0.4, rtw.Dialectric(1 / 1.5)))
    if metal: world.add(rtw.Sphere((1, 0, -1), 0.5, rtw.Metal((0.8, 0.6, 0.2), 0.3)))
    if invisible: world.add(rtw.Sphere((0.3, 0.2, -0.8), 0.1, rtw.INVISIBLE))
    li = [rtw.Sphere((0, 0, -1.2), 0.6 if inside_light else 0.2)] if True else []
    if two_lights: li.append(rtw.Sphere((1, 1, 0), 0.2))
    return rtw.flatten(world, rtw.HittableList(li))

def run(soa, defocus):
    b = rtw.CameraBuilder().with_image_width(40).with_image_height(30).with_samples_per_pixel(6) \
        .with_max_depth(20).with_lookfrom((0, 0.3, 1)).with_lookat((0, 0, -1)) \
        .with_focus_dist(2.0).with_background((0.7, 0.8, 1.0))
    if defocus: b.with_defocus_angle(0.05)
    cam = b.build()
    with rtw.Renderer(precision=rtw.RTW_F64) as r:
        r.set_scene(soa); g = r.render(cam, 5); chunk = r.stats.chunk; segs = r.stats.segments
    ocam = O.Camera()
    for n, _ in O.Camera._fields_: setattr(ocam, n, getattr(cam.raw, n))
    ref, st = O.render(ocam, O.Scene(**soa.__dict__), 5, chunk=chunk)
    ng, nr = np.isnan(g).any(-1), np.isnan(ref).any(-1)
    ok = ~(ng | nr)
    ex = (g == ref).all(-1)[ok].mean()
    return ng.sum(), nr.sum(), ex, segs, st.segments

base = dict(plane=True, nested=True, invisible=True, inside_light=True, two_lights=True, metal=True)
print("all", run(scene(**base), True))
print("no defocus", run(scene(**base), False))
for k in base:
    kw = dict(base); kw[k] = False
    print("no", k, run(scene(**kw), True))
