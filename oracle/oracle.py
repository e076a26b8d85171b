"""ctypes wrapper of the CPU oracle (oracle/liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg -- never by the product package.  See
oracle/rtw_oracle.h for what is restated from which reference file:line and
why parity against the Rust reference binary itself is unpinned.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from dataclasses import dataclass

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")

LAMBERTIAN, METAL, DIELECTRIC, INVISIBLE, DIFFUSE_LIGHT = 0, 1, 2, 3, 4
TEX_SOLID, TEX_CHECKER, TEX_NOISE = 0, 1, 2
LIGHTS_BVH_LEAF = 1


class ReferencePanic(RuntimeError):
    """The render reached a point where the reference panics (stats.panic_*)."""

    def __init__(self, msg, stats):
        super().__init__(msg)
        self.stats = stats
ACCEL_BRUTE, ACCEL_BVH_REF, ACCEL_BVH_CACHED = 0, 1, 2

_u32p = C.POINTER(C.c_uint32)
_f64p = C.POINTER(C.c_double)
_u64p = C.POINTER(C.c_uint64)


class Camera(C.Structure):
    _fields_ = [
        ("image_width", C.c_uint32), ("image_height", C.c_uint32),
        ("samples_per_pixel", C.c_uint32), ("max_depth", C.c_uint32),
        ("background", C.c_double * 3), ("defocus_angle", C.c_double),
        ("center", C.c_double * 3), ("pixel00_loc", C.c_double * 3),
        ("pixel_delta_u", C.c_double * 3), ("pixel_delta_v", C.c_double * 3),
        ("defocus_disk_u", C.c_double * 3), ("defocus_disk_v", C.c_double * 3),
    ]


class CameraBuilder(C.Structure):
    _fields_ = [
        ("has_aspect_ratio", C.c_int), ("has_image_width", C.c_int), ("has_image_height", C.c_int),
        ("aspect_ratio", C.c_double), ("image_width", C.c_uint32), ("image_height", C.c_uint32),
        ("samples_per_pixel", C.c_uint32), ("max_depth", C.c_uint32),
        ("background", C.c_double * 3), ("vfov", C.c_double),
        ("lookfrom", C.c_double * 3), ("lookat", C.c_double * 3), ("vup", C.c_double * 3),
        ("defocus_angle", C.c_double), ("focus_dist", C.c_double),
    ]


class _Scene(C.Structure):
    _fields_ = [
        ("n_spheres", C.c_uint32), ("spheres", _f64p), ("sphere_mat", _u32p),
        ("n_planes", C.c_uint32), ("planes", _f64p), ("plane_mat", _u32p),
        ("n_materials", C.c_uint32), ("mat_type", _u32p), ("mat_params", _f64p),
        ("n_lights", C.c_uint32), ("lights", _f64p),
        ("n_quads", C.c_uint32), ("quads", _f64p), ("quad_mat", _u32p),
        ("n_light_quads", C.c_uint32), ("light_quads", _f64p), ("light_kinds", _u32p),
        ("n_boxes", C.c_uint32), ("boxes", _f64p), ("box_mat", _u32p),
        ("mat_tex", _u32p), ("n_textures", C.c_uint32), ("tex_type", _u32p), ("tex_params", _f64p),
        ("tex_refs", _u32p), ("n_perlin", C.c_uint32), ("perlin_vec", _f64p), ("perlin_perm", _u32p),
        ("n_light_other", C.c_uint32), ("light_flags", C.c_uint32),
    ]


class Stats(C.Structure):
    _fields_ = [("samples", C.c_uint64), ("segments", C.c_uint64),
                ("lambertian", C.c_uint64), ("nan_samples", C.c_uint64),
                ("panic_plane_uv", C.c_uint64), ("panic_no_lights", C.c_uint64)]


@dataclass
class Scene:
    """Flat SoA scene (the same layout the C-ABI's rtw_scene carries)."""
    spheres: np.ndarray      # (n, 4) cx, cy, cz, r
    sphere_mat: np.ndarray   # (n,) uint32
    planes: np.ndarray       # (m, 6) px, py, pz, nx, ny, nz
    plane_mat: np.ndarray    # (m,) uint32
    mat_type: np.ndarray     # (k,) uint32
    mat_params: np.ndarray   # (k, 5) albedo rgb, fuzz, ior
    lights: np.ndarray       # (l, 4)
    quads: np.ndarray = None         # (q, 9) Q, u, v
    quad_mat: np.ndarray = None      # (q,) uint32
    light_quads: np.ndarray = None   # (lq, 9)
    light_kinds: np.ndarray = None   # (l + lq + lo,) 0 sphere / 1 quad / 2 Hittable defaults, list order;
                                     # None = spheres first
    boxes: np.ndarray = None         # (b, 18) Cuboid p, q, rotation R (row-major), translation T
    box_mat: np.ndarray = None       # (b,) uint32
    mat_tex: np.ndarray = None       # (k,) texture id per material; None = SolidColour albedos
    tex_type: np.ndarray = None      # (t,) TEX_SOLID / TEX_CHECKER / TEX_NOISE
    tex_params: np.ndarray = None    # (t, 4) solid rgb | checker inv_scale [3] | noise scale [3]
    tex_refs: np.ndarray = None      # (t, 2) checker even/odd ids | noise perlin id
    perlin_vec: np.ndarray = None    # (p, 256, 3) Perlin::rand_vec
    perlin_perm: np.ndarray = None   # (p, 3, 256) perm_x, perm_y, perm_z
    n_light_other: int = 0
    light_flags: int = 0             # LIGHTS_BVH_LEAF


_lib = None


def build(force: bool = False) -> str:
    """Compile liboracle.so with oracle/Makefile (gcc)."""
    if force or not os.path.exists(LIB_PATH):
        subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        L.rtwo_camera_build.argtypes = [C.POINTER(CameraBuilder), C.POINTER(Camera)]
        L.rtwo_render.argtypes = [C.POINTER(Camera), C.POINTER(_Scene), C.c_uint64, C.c_uint32,
                                  C.c_int, C.c_int, C.c_uint32, C.c_uint32, C.c_uint32,
                                  C.c_uint32, C.c_uint32, _f64p, C.POINTER(Stats)]
        L.rtwo_trace_sample.argtypes = [C.POINTER(Camera), C.POINTER(_Scene), C.c_uint64,
                                        C.c_uint32, C.c_uint32, C.c_uint32, _f64p, C.POINTER(Stats)]
        L.rtwo_scene_simple.argtypes = [C.c_uint64, C.c_int, C.c_uint32, _f64p, _u32p, _u32p,
                                        _f64p, _u32p, _u32p, C.c_uint32, _u32p, _f64p, _u32p,
                                        C.c_uint32, _f64p, _u32p]
        L.rtwo_rng_seed.argtypes = [C.c_uint64, C.c_uint64, C.c_uint64, _u64p]
        L.rtwo_rng_next.argtypes = [_u64p]
        L.rtwo_rng_next.restype = C.c_uint64
        for name in ("rtwo_rand_std", "rtwo_rand_open01"):
            getattr(L, name).argtypes = [_u64p]
            getattr(L, name).restype = C.c_double
        L.rtwo_rand_uniform_incl.argtypes = [_u64p, C.c_double, C.c_double]
        L.rtwo_rand_uniform_incl.restype = C.c_double
        L.rtwo_rand_index.argtypes = [_u64p, C.c_uint32]
        L.rtwo_rand_index.restype = C.c_uint32
        L.rtwo_sincos_2pi.argtypes = [C.c_double, _f64p, _f64p]
        L.rtwo_sphere_hit.argtypes = [_f64p, _f64p, _f64p, C.c_double, C.c_double, _f64p, _f64p,
                                      C.POINTER(C.c_int)]
        L.rtwo_plane_hit.argtypes = L.rtwo_sphere_hit.argtypes
        L.rtwo_aabb_hit.argtypes = [_f64p, _f64p, _f64p, C.c_double, C.c_double]
        L.rtwo_sphere_pdf_value.argtypes = [_f64p, _f64p, _f64p]
        L.rtwo_sphere_pdf_value.restype = C.c_double
        L.rtwo_onb.argtypes = [_f64p, _f64p, _f64p, _f64p]
        L.rtwo_reflectance.argtypes = [C.c_double, C.c_double]
        L.rtwo_reflectance.restype = C.c_double
        L.rtwo_reflect.argtypes = [_f64p, _f64p, _f64p]
        L.rtwo_refract.argtypes = [_f64p, _f64p, C.c_double, _f64p]
        L.rtwo_unit_sphere.argtypes = [_u64p, _f64p]
        L.rtwo_cosine_hemisphere.argtypes = [_u64p, _f64p]
        L.rtwo_sphere_random.argtypes = [_f64p, _f64p, _u64p, _f64p]
        L.rtwo_bvh_stats.argtypes = [C.POINTER(_Scene), _u32p, _u32p, _u32p]
        L.rtwo_quad_hit.argtypes = [_f64p, _f64p, _f64p, C.c_double, C.c_double, _f64p]
        L.rtwo_quad_pdf_value.argtypes = [_f64p, _f64p, _f64p]
        L.rtwo_quad_pdf_value.restype = C.c_double
        L.rtwo_quad_random.argtypes = [_f64p, _f64p, _u64p, _f64p]
        L.rtwo_quad_aabb.argtypes = [_f64p, _f64p]
        L.rtwo_box_hit.argtypes = [_f64p, _f64p, _f64p, C.c_double, C.c_double, _f64p]
        L.rtwo_box_aabb.argtypes = [_f64p, _f64p]
        L.rtwo_trace_path.argtypes = [C.POINTER(Camera), C.POINTER(_Scene), C.c_uint64, C.c_uint32,
                                      C.c_uint32, C.c_uint32, C.c_int, _f64p, C.POINTER(Stats), _f64p,
                                      C.c_uint32]
        L.rtwo_trace_path.restype = C.c_uint32
        L.rtwo_world_hit.argtypes = [C.POINTER(_Scene), C.c_int, _f64p, _f64p, _f64p]
        L.rtwo_sin.argtypes = [C.c_double]
        L.rtwo_sin.restype = C.c_double
        L.rtwo_sphere_uv.argtypes = [_f64p, _f64p]
        L.rtwo_plane_uv.argtypes = [_f64p, _f64p, _f64p]
        L.rtwo_perlin_noise.argtypes = [_f64p, _u32p, _f64p]
        L.rtwo_perlin_noise.restype = C.c_double
        L.rtwo_perlin_turb.argtypes = [_f64p, _u32p, _f64p, C.c_int]
        L.rtwo_perlin_turb.restype = C.c_double
        L.rtwo_texture_colour.argtypes = [C.POINTER(_Scene), C.c_uint32, C.c_double, C.c_double, _f64p, _f64p]
        _lib = L
    return _lib


def _p(a, t):
    return a.ctypes.data_as(t)


def arr(x, n=3):
    return (C.c_double * n)(*x)


def dptr(a):
    a = np.ascontiguousarray(a, dtype=np.float64)
    return a, _p(a, _f64p)


def make_builder(**kw) -> CameraBuilder:
    """CameraBuilder::new() defaults (camera.rs:45-60) plus overrides."""
    b = CameraBuilder()
    b.samples_per_pixel = kw.get("samples_per_pixel", 10)
    b.max_depth = kw.get("max_depth", 10)
    b.background = arr(kw.get("background", (0.0, 0.0, 0.0)))
    b.vfov = kw.get("vfov", 90.0)
    b.lookfrom = arr(kw.get("lookfrom", (0.0, 0.0, 0.0)))
    b.lookat = arr(kw.get("lookat", (0.0, 0.0, -1.0)))
    b.vup = arr(kw.get("vup", (0.0, 1.0, 0.0)))
    b.defocus_angle = kw.get("defocus_angle", 0.0)
    b.focus_dist = kw.get("focus_dist", 10.0)
    if kw.get("aspect_ratio") is not None:
        b.has_aspect_ratio, b.aspect_ratio = 1, kw["aspect_ratio"]
    if kw.get("image_width") is not None:
        b.has_image_width, b.image_width = 1, kw["image_width"]
    if kw.get("image_height") is not None:
        b.has_image_height, b.image_height = 1, kw["image_height"]
    return b


def camera_build(**kw) -> Camera:
    cam = Camera()
    lib().rtwo_camera_build(C.byref(make_builder(**kw)), C.byref(cam))
    return cam


def camera_dict(cam: Camera) -> dict:
    out = {}
    for name, _ in Camera._fields_:
        v = getattr(cam, name)
        out[name] = list(v) if not isinstance(v, (int, float)) else v
    return out


def scene_simple(seed: int, n: int = 11) -> Scene:
    """scenes::simple restated (scenes/src/lib.rs:155-233)."""
    cells = (2 * n) * (2 * n)
    ms, mm, ml = cells + 3, cells + 4, cells + 1
    sph = np.zeros((ms, 4)); smat = np.zeros(ms, np.uint32)
    pl = np.zeros((1, 6)); plm = np.zeros(1, np.uint32)
    mt = np.zeros(mm, np.uint32); mp = np.zeros((mm, 5))
    li = np.zeros((ml, 4))
    ns, npl, nm, nl = (C.c_uint32() for _ in range(4))
    rc = lib().rtwo_scene_simple(
        C.c_uint64(seed & 0xFFFFFFFFFFFFFFFF), n, ms, _p(sph, _f64p), _p(smat, _u32p), C.byref(ns),
        _p(pl, _f64p), _p(plm, _u32p), C.byref(npl), mm, _p(mt, _u32p), _p(mp, _f64p), C.byref(nm),
        ml, _p(li, _f64p), C.byref(nl))
    assert rc == 0
    return Scene(sph[: ns.value].copy(), smat[: ns.value].copy(), pl[: npl.value].copy(),
                 plm[: npl.value].copy(), mt[: nm.value].copy(), mp[: nm.value].copy(),
                 li[: nl.value].copy())


def simple_camera_kw(n: int = 11) -> dict:
    """The camera scenes::simple hands back (scenes/src/lib.rs:219-226), with
    bin/src/main.rs:72-79's vfov override.  For n > 11 the camera is pulled
    back proportionally (the C3/C5 synthetic scenes of SURVEY.md §8d)."""
    k = max(1.0, n / 11.0)
    lookfrom = (10.0 * k, 5.0 * k, 10.0 * k)
    lookat = (0.0, 0.0, 0.0)
    focus = float(np.sqrt(sum((a - b) ** 2 for a, b in zip(lookfrom, lookat))))
    # (lookfrom - lookat).length() in f64: restate the reference's dot order
    d = [a - b for a, b in zip(lookfrom, lookat)]
    focus = float(np.sqrt((d[0] * d[0] + d[1] * d[1]) + d[2] * d[2]))
    return dict(lookfrom=lookfrom, lookat=lookat, focus_dist=focus, vfov=40.0,
                background=(1.0, 1.0, 1.0))


def _scene_struct(sc: Scene):
    keep = []

    def f(a, cols):
        a = np.ascontiguousarray(np.asarray(a, dtype=np.float64).reshape(-1, cols))
        keep.append(a)
        return _p(a, _f64p)

    def u(a):
        a = np.ascontiguousarray(np.asarray(a, dtype=np.uint32).reshape(-1))
        keep.append(a)
        return _p(a, _u32p)

    quads = np.zeros((0, 9)) if sc.quads is None else sc.quads
    qmat = np.zeros(0, np.uint32) if sc.quad_mat is None else sc.quad_mat
    lq = np.zeros((0, 9)) if sc.light_quads is None else sc.light_quads
    s = _Scene(len(sc.sphere_mat), f(sc.spheres, 4), u(sc.sphere_mat),
               len(sc.plane_mat), f(sc.planes, 6), u(sc.plane_mat),
               len(sc.mat_type), u(sc.mat_type), f(sc.mat_params, 5),
               len(np.asarray(sc.lights).reshape(-1, 4)), f(sc.lights, 4),
               len(np.asarray(qmat).reshape(-1)), f(quads, 9), u(qmat),
               len(np.asarray(lq).reshape(-1, 9)), f(lq, 9),
               None if sc.light_kinds is None else u(sc.light_kinds),
               0 if sc.box_mat is None else len(np.asarray(sc.box_mat).reshape(-1)),
               f(np.zeros((0, 18)) if sc.boxes is None else sc.boxes, 18),
               u(np.zeros(0, np.uint32) if sc.box_mat is None else sc.box_mat),
               None if sc.mat_tex is None else u(sc.mat_tex),
               0 if sc.tex_type is None else len(np.asarray(sc.tex_type).reshape(-1)),
               u(np.zeros(0) if sc.tex_type is None else sc.tex_type),
               f(np.zeros((0, 4)) if sc.tex_params is None else sc.tex_params, 4),
               u(np.zeros(0) if sc.tex_refs is None else sc.tex_refs),
               0 if sc.perlin_vec is None else len(np.asarray(sc.perlin_vec).reshape(-1, 768)),
               f(np.zeros((0, 768)) if sc.perlin_vec is None else sc.perlin_vec, 768),
               u(np.zeros(0) if sc.perlin_perm is None else sc.perlin_perm),
               int(sc.n_light_other), int(sc.light_flags))
    return s, keep


def render(cam: Camera, sc: Scene, seed: int, *, chunk: int = 0, accel: int = ACCEL_BRUTE,
           threads: int = 0, rows=None, cols=None, out=None, allow_panic: bool = False):
    """Camera::render restated.  Returns (sums[H, W, 3] float64, Stats).
    rows = (begin, end, step); cols = (begin, end)."""
    H, W = cam.image_height, cam.image_width
    if out is None:
        out = np.zeros((H, W, 3), np.float64)
    rb, re, rs = rows if rows is not None else (0, H, 1)
    cb, ce = cols if cols is not None else (0, W)
    if threads <= 0:
        threads = min(os.cpu_count() or 1, 16)
    s, keep = _scene_struct(sc)
    st = Stats()
    rc = lib().rtwo_render(C.byref(cam), C.byref(s), C.c_uint64(seed & 0xFFFFFFFFFFFFFFFF), chunk,
                           accel, threads, rb, re, rs, cb, ce, _p(out, _f64p), C.byref(st))
    del keep
    if rc == -2 and not allow_panic:
        raise ReferencePanic(f"the reference panics on this render (plane UV: {st.panic_plane_uv}, "
                             f"empty light list: {st.panic_no_lights} samples)", st)
    if rc not in (0, -2):
        raise ValueError("oracle render rejected the scene")
    return out, st


def trace_sample(cam: Camera, sc: Scene, seed: int, i: int, j: int, s: int):
    st = Stats()
    rgb = np.zeros(3)
    ss, keep = _scene_struct(sc)
    lib().rtwo_trace_sample(C.byref(cam), C.byref(ss), C.c_uint64(seed), i, j, s, _p(rgb, _f64p),
                            C.byref(st))
    del keep
    return rgb, st


def trace_path(cam: Camera, sc: Scene, seed: int, i: int, j: int, s: int, accel=ACCEL_BRUTE, cap=64):
    """(rgb, [segments x {o xyz, d xyz, id, t}]) of one sample (debugging / KATs)."""
    st = Stats()
    rgb = np.zeros(3)
    path = np.zeros((cap, 8))
    ss, keep = _scene_struct(sc)
    n = lib().rtwo_trace_path(C.byref(cam), C.byref(ss), C.c_uint64(seed), i, j, s, accel,
                              _p(rgb, _f64p), C.byref(st), _p(path, _f64p), cap)
    del keep
    return rgb, path[:min(n, cap)]


def bvh_stats(sc: Scene):
    s, keep = _scene_struct(sc)
    a, b, c = C.c_uint32(), C.c_uint32(), C.c_uint32()
    lib().rtwo_bvh_stats(C.byref(s), C.byref(a), C.byref(b), C.byref(c))
    return a.value, b.value, c.value


class Rng:
    """The build's per-(pixel, sample) RNG stream, for KATs."""

    def __init__(self, seed=0, pixel=0, sample=0):
        self.st = (C.c_uint64 * 4)()
        lib().rtwo_rng_seed(C.c_uint64(seed), C.c_uint64(pixel), C.c_uint64(sample), self.st)

    def next_u64(self):
        return lib().rtwo_rng_next(self.st)

    def std(self):
        return lib().rtwo_rand_std(self.st)

    def open01(self):
        return lib().rtwo_rand_open01(self.st)

    def uniform_incl(self, lo, hi):
        return lib().rtwo_rand_uniform_incl(self.st, lo, hi)

    def index(self, n):
        return lib().rtwo_rand_index(self.st, n)


# ---- Quad (quadrilateral.rs) KAT entry points
def quad_hit(quad, o, d, tmin=2.220446049250313e-16, tmax=float("inf")):
    """(t, alpha, beta, normal[3]) or None."""
    out = (C.c_double * 6)()
    hit = lib().rtwo_quad_hit(arr(quad, 9), arr(o), arr(d), tmin, tmax, out)
    return (out[0], out[1], out[2], tuple(out[3:6])) if hit else None


def quad_pdf_value(quad, o, d):
    return lib().rtwo_quad_pdf_value(arr(quad, 9), arr(o), arr(d))


def quad_random(quad, o, rng: "Rng"):
    out = (C.c_double * 3)()
    lib().rtwo_quad_random(arr(quad, 9), arr(o), rng.st, out)
    return tuple(out)


def quad_aabb(quad):
    out = (C.c_double * 6)()
    lib().rtwo_quad_aabb(arr(quad, 9), out)
    return tuple(out[:3]), tuple(out[3:])


# ---- Transformed<Cuboid> KAT entry points
def box_hit(box, o, d, tmin=2.220446049250313e-16, tmax=float("inf")):
    """(t, world point[3], object-space normal[3], front) or None."""
    out = (C.c_double * 8)()
    hit = lib().rtwo_box_hit(arr(box, 18), arr(o), arr(d), tmin, tmax, out)
    return (out[0], tuple(out[1:4]), tuple(out[4:7]), bool(out[7])) if hit else None


def box_aabb(box):
    out = (C.c_double * 6)()
    lib().rtwo_box_aabb(arr(box, 18), out)
    return tuple(out[:3]), tuple(out[3:])


def transform_compose(*steps):
    """Transformation::then chain (geometry/src/transformations.rs:97-108):
    steps are ('translate', (x, y, z)) or ('rotate', angle_deg, axis 0/1/2),
    applied in order; returns (R 3x3 list, T 3-list) as the reference's
    f64 arithmetic computes them."""
    R = [[1.0, 0.0, 0.0], [0.0, 1.0, 0.0], [0.0, 0.0, 1.0]]
    T = [0.0, 0.0, 0.0]
    for st in steps:
        if st[0] == "translate":
            bR, bT = [[1.0, 0.0, 0.0], [0.0, 1.0, 0.0], [0.0, 0.0, 1.0]], list(map(float, st[1]))
        else:
            bR, bT = rotation_matrix(st[1], st[2]), [0.0, 0.0, 0.0]
        # apply: rotation = b.R * self.R, translation = b.T + b.R * self.T
        nR = [[_dot(bR[i], [R[0][j], R[1][j], R[2][j]]) for j in range(3)] for i in range(3)]
        bRT = [_dot(bR[i], T) for i in range(3)]
        T = [bT[i] + bRT[i] for i in range(3)]
        R = nR
    return R, T


def _dot(a, b):
    return (a[0] * b[0] + a[1] * b[1]) + a[2] * b[2]


def rotation_matrix(angle_deg, axis):
    """geometry::transformations::rotation (non-euclid), angle.to_radians()
    = angle * (PI / 180) as Rust's f64::to_radians."""
    import math
    a = angle_deg * (math.pi / 180.0)
    c, s = math.cos(a), math.sin(a)
    if axis == 0:
        return [[1.0, 0.0, 0.0], [0.0, c, -s], [0.0, s, c]]
    if axis == 1:
        return [[c, 0.0, s], [0.0, 1.0, 0.0], [-s, 0.0, c]]
    return [[c, -s, 0.0], [s, c, 0.0], [0.0, 0.0, 1.0]]


def world_hit(sc: Scene, o, d, accel=ACCEL_BRUTE):
    """(object id, t, p, normal, front) of world.hit, or (-1, ...)."""
    s, keep = _scene_struct(sc)
    out = (C.c_double * 8)()
    k = lib().rtwo_world_hit(C.byref(s), accel, arr(o), arr(d), out)
    del keep
    return k, out[0], tuple(out[1:4]), tuple(out[4:7]), bool(out[7])


# ---- texture KAT entry points
def sin(x):
    return lib().rtwo_sin(float(x))


def sphere_uv(n):
    out = (C.c_double * 2)()
    lib().rtwo_sphere_uv(arr(n), out)
    return out[0], out[1]


def plane_uv(plane, p):
    out = (C.c_double * 2)()
    lib().rtwo_plane_uv(arr(plane, 6), arr(p), out)
    return out[0], out[1]


def perlin_noise(vec, perm, p):
    v, vp = dptr(np.asarray(vec).reshape(-1))
    pm = np.ascontiguousarray(np.asarray(perm, np.uint32).reshape(-1))
    return lib().rtwo_perlin_noise(vp, _p(pm, _u32p), arr(p))


def perlin_turb(vec, perm, p, depth=7):
    v, vp = dptr(np.asarray(vec).reshape(-1))
    pm = np.ascontiguousarray(np.asarray(perm, np.uint32).reshape(-1))
    return lib().rtwo_perlin_turb(vp, _p(pm, _u32p), arr(p), depth)


def texture_colour(sc: Scene, tid, u, v, p):
    s, keep = _scene_struct(sc)
    out = (C.c_double * 3)()
    lib().rtwo_texture_colour(C.byref(s), tid, u, v, arr(p), out)
    del keep
    return tuple(out)
