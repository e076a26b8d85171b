"""ray_tracing_weekend_amd -- MI355X (gfx950) drop-in for the reference's
per-pixel / per-sample ray_colour loop (N9199/ray_tracing_weekend).

Python mirror of the reference's interface for this path, over the C-ABI in
include/rtw.h (librtw.so: hand-written HIP kernels + C++ host mirror):

    world, lights, builder = scenes.simple(seed)          # scenes/src/lib.rs:155-233
    cam = builder.with_image_width(400).with_image_height(225) \
                 .with_samples_per_pixel(100).with_max_depth(50).build()
    sums = cam.render(world, lights)                      # shared/src/camera.rs:295-297
    write_ppm("image.ppm", sums, cam.samples_per_pixel)   # bin/src/main.rs:89-104

`render` returns per-pixel SUMS (not means) as a float64 array [H, W, 3] with
row j = 0 at the BOTTOM, like render_internal's Vec<Vec<Colour>>.
"""
from __future__ import annotations

import ctypes as C
import math
from dataclasses import dataclass, field

import numpy as np

from . import _capi
from ._capi import (RTW_ACCEL_AUTO, RTW_ACCEL_BRUTE, RTW_ACCEL_BVH, RTW_DIELECTRIC, RTW_F32,
                    RTW_F64, RTW_INVISIBLE, RTW_LAMBERTIAN, RTW_METAL, RTW_DIFFUSE_LIGHT, RTW_TEX_SOLID,
                    RTW_TEX_CHECKER, RTW_TEX_NOISE, RTW_LIGHT_SPHERE, RTW_LIGHT_QUAD, RTW_LIGHT_DEFAULT,
                    RTW_LIGHTS_BVH_LEAF)

__all__ = [
    "Material", "Lambertian", "Metal", "Dialectric", "DiffuseLight", "INVISIBLE", "Sphere", "Plane",
    "Quad", "Cuboid", "Transformation", "translation", "rotation", "SolidColour", "CheckerTexture",
    "NoiseTexture", "Perlin", "HittableList", "BoundedVolumeHierarchy", "SceneSoA", "flatten",
    "CameraBuilder", "Camera", "Renderer", "scenes", "encode_rgb8", "write_ppm", "RenderError",
    "RTW_F32", "RTW_F64",
]

_lib = _capi.load()   # raises if librtw.so is missing: there is no CPU fallback


class RenderError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"{msg} (rtw error {code})")
        self.code = code


# ---------------------------------------------------------------- textures
class Perlin:                                # perlin.rs:13-58
    """Perlin::new with the build's seeded RNG (the reference draws the
    tables from thread_rng): rand_vec (256 x 3) and perm (3 x 256)."""

    def __init__(self, seed: int = 0x5EED0001):
        self.rand_vec = np.zeros((256, 3), np.float64)
        self.perm = np.zeros((3, 256), np.uint32)
        rc = _lib.rtw_perlin_generate(C.c_uint64(seed & 0xFFFFFFFFFFFFFFFF),
                                      self.rand_vec.ctypes.data_as(_capi._f64p),
                                      self.perm.ctypes.data_as(_capi._u32p))
        if rc != 0:
            raise RenderError(rc, "rtw_perlin_generate failed")


@dataclass(frozen=True, eq=False)
class SolidColour:                           # texture.rs:15-22
    colour: tuple


@dataclass(frozen=True, eq=False)
class CheckerTexture:                        # texture.rs:24-55
    even: object
    odd: object
    inv_scale: float

    @staticmethod
    def new(even, odd, scale: float) -> "CheckerTexture":
        return CheckerTexture(even, odd, 1.0 / float(scale))          # scale.recip()

    @staticmethod
    def new_with_colours(even, odd, scale: float) -> "CheckerTexture":
        return CheckerTexture.new(SolidColour(tuple(map(float, even))), SolidColour(tuple(map(float, odd))), scale)


@dataclass(frozen=True, eq=False)
class NoiseTexture:                          # texture.rs:57-102
    scale: float
    noise: Perlin

    @staticmethod
    def new(scale: float, seed: int = 0x5EED0001) -> "NoiseTexture":
        return NoiseTexture(float(scale), Perlin(seed))


_TEXTURES = (SolidColour, CheckerTexture, NoiseTexture)


# ---------------------------------------------------------------- materials
@dataclass(frozen=True)
class Material:
    type: int
    albedo: tuple = (0.0, 0.0, 0.0)
    fuzz: float = 0.0
    ior: float = 0.0
    texture: object = None                   # Lambertian / DiffuseLight texture; None = SolidColour(albedo)


def Lambertian(albedo):                      # material.rs:347-355 (new / new_with_colour)
    if isinstance(albedo, _TEXTURES):
        return Material(RTW_LAMBERTIAN, texture=albedo)
    return Material(RTW_LAMBERTIAN, tuple(map(float, albedo)))


def Metal(albedo, fuzz):                     # material.rs:378-406
    return Material(RTW_METAL, tuple(map(float, albedo)), float(fuzz))


def Dialectric(index_of_refraction):         # material.rs:423-455
    return Material(RTW_DIELECTRIC, (1.0, 1.0, 1.0), 0.0, float(index_of_refraction))


INVISIBLE = Material(RTW_INVISIBLE)          # material.rs:321-325


def DiffuseLight(colour):                    # material.rs:490-514 (new / new_with_colour)
    if isinstance(colour, _TEXTURES):
        return Material(RTW_DIFFUSE_LIGHT, texture=colour)
    return Material(RTW_DIFFUSE_LIGHT, tuple(map(float, colour)))


@dataclass(frozen=True)
class Sphere:                                # entities/sphere.rs:24-47
    center: tuple
    radius: float
    mat: Material = INVISIBLE


@dataclass(frozen=True)
class Plane:                                 # entities/plane.rs:20-38 (normal normalized)
    point: tuple
    normal: tuple
    mat: Material = INVISIBLE

    def __post_init__(self):
        n = [float(v) for v in self.normal]
        ln = np.sqrt((n[0] * n[0] + n[1] * n[1]) + n[2] * n[2])
        object.__setattr__(self, "normal", (n[0] / ln, n[1] / ln, n[2] / ln))


@dataclass(frozen=True)
class Quad:                                  # entities/quadrilateral.rs:21-56 (Quad::new(Q, u, v, mat))
    q: tuple
    u: tuple
    v: tuple
    mat: Material = INVISIBLE


@dataclass(frozen=True)
class Transformation:
    """geometry::transformations::Transformation (non-euclid build): point ->
    R p + T.  `then` composes like the reference (transformations.rs:97-108)."""
    R: tuple = ((1.0, 0.0, 0.0), (0.0, 1.0, 0.0), (0.0, 0.0, 1.0))
    T: tuple = (0.0, 0.0, 0.0)

    def then(self, b: "Transformation") -> "Transformation":
        def dot(u, v):
            return (u[0] * v[0] + u[1] * v[1]) + u[2] * v[2]
        cols = [[self.R[0][j], self.R[1][j], self.R[2][j]] for j in range(3)]
        R = tuple(tuple(dot(b.R[i], cols[j]) for j in range(3)) for i in range(3))
        bRT = [dot(b.R[i], self.T) for i in range(3)]
        return Transformation(R, tuple(b.T[i] + bRT[i] for i in range(3)))


def translation(v) -> Transformation:        # Translation3 = Vec3 -> Transformation (vec3.rs:11)
    return Transformation(T=tuple(map(float, v)))


def rotation(angle_deg: float, axis: int) -> Transformation:   # transformations.rs:37-58 (axis 0/1/2 = X/Y/Z)
    a = float(angle_deg) * (math.pi / 180.0)                  # f64::to_radians
    c, s = math.cos(a), math.sin(a)                           # libm, as f64::cos / f64::sin
    R = [((1.0, 0.0, 0.0), (0.0, c, -s), (0.0, s, c)),
         ((c, 0.0, s), (0.0, 1.0, 0.0), (-s, 0.0, c)),
         ((c, -s, 0.0), (s, c, 0.0), (0.0, 0.0, 1.0))][axis]
    return Transformation(R=R)


@dataclass(frozen=True)
class Cuboid:                                # entities/cuboid.rs:26-47, Cuboid::new(p, q, mat)
    p: tuple
    q: tuple
    mat: Material = INVISIBLE
    xform: Transformation = Transformation()

    def transform(self, t: Transformation) -> "Cuboid":
        """Transformable::transform (transformations.rs:187-211): the
        transformations compose in call order."""
        return Cuboid(self.p, self.q, self.mat, self.xform.then(t))


class HittableList:                          # hittable_collections/hittable_list.rs:247-294
    def __init__(self, objects=()):
        self.objects = []
        for o in objects:
            self.add(o)

    def add(self, obj):
        if not isinstance(obj, (Sphere, Plane, Quad, Cuboid)):
            raise TypeError("only Sphere, Plane, Quad and (transformed) Cuboid are in this build's scope")
        self.objects.append(obj)

    def __len__(self):
        return len(self.objects)


class BoundedVolumeHierarchy(HittableList):  # hittable_collections/bvh.rs:106-143 (::from(list))
    """The reference's BVH over a list: as the world it gives the list's
    closest hit (the device builds its own tree); as a light list its
    pdf_value is (sum / n * n) / n for a leaf of <= 5 entries (bvh.rs:67-76,
    191-194).  Deeper BVH light lists are outside this build (their
    aux_random indexing, bvh.rs:78-92, is inconsistent)."""

    def __init__(self, lst=()):
        super().__init__(lst.objects if isinstance(lst, HittableList) else lst)


@dataclass
class SceneSoA:
    """Flattened world + lights in the C-ABI's struct-of-arrays layout."""
    spheres: np.ndarray = field(default_factory=lambda: np.zeros((0, 4)))
    sphere_mat: np.ndarray = field(default_factory=lambda: np.zeros(0, np.uint32))
    planes: np.ndarray = field(default_factory=lambda: np.zeros((0, 6)))
    plane_mat: np.ndarray = field(default_factory=lambda: np.zeros(0, np.uint32))
    mat_type: np.ndarray = field(default_factory=lambda: np.zeros(0, np.uint32))
    mat_params: np.ndarray = field(default_factory=lambda: np.zeros((0, 5)))
    lights: np.ndarray = field(default_factory=lambda: np.zeros((0, 4)))
    quads: np.ndarray = field(default_factory=lambda: np.zeros((0, 9)))
    quad_mat: np.ndarray = field(default_factory=lambda: np.zeros(0, np.uint32))
    light_quads: np.ndarray = field(default_factory=lambda: np.zeros((0, 9)))
    light_kinds: np.ndarray = None          # list order: 0 sphere / 1 quad; None = spheres first
    boxes: np.ndarray = field(default_factory=lambda: np.zeros((0, 18)))
    box_mat: np.ndarray = field(default_factory=lambda: np.zeros(0, np.uint32))
    mat_tex: np.ndarray = None              # texture id per material; None = SolidColour albedos
    tex_type: np.ndarray = field(default_factory=lambda: np.zeros(0, np.uint32))
    tex_params: np.ndarray = field(default_factory=lambda: np.zeros((0, 4)))
    tex_refs: np.ndarray = field(default_factory=lambda: np.zeros((0, 2), np.uint32))
    perlin_vec: np.ndarray = field(default_factory=lambda: np.zeros((0, 256, 3)))
    perlin_perm: np.ndarray = field(default_factory=lambda: np.zeros((0, 3, 256), np.uint32))
    n_light_other: int = 0
    light_flags: int = 0

    def as_c(self):
        """(rtw_scene, keepalive) -- the struct points into these arrays."""
        keep = []

        def f(a, cols):
            a = np.ascontiguousarray(np.asarray(a, np.float64).reshape(-1, cols))
            keep.append(a)
            return a.ctypes.data_as(_capi._f64p)

        def u(a):
            a = np.ascontiguousarray(np.asarray(a, np.uint32).reshape(-1))
            keep.append(a)
            return a.ctypes.data_as(_capi._u32p)

        s = _capi.rtw_scene(len(self.sphere_mat), f(self.spheres, 4), u(self.sphere_mat),
                            len(self.plane_mat), f(self.planes, 6), u(self.plane_mat),
                            len(self.mat_type), u(self.mat_type), f(self.mat_params, 5),
                            len(np.asarray(self.lights).reshape(-1, 4)), f(self.lights, 4),
                            len(self.quad_mat), f(self.quads, 9), u(self.quad_mat),
                            len(np.asarray(self.light_quads).reshape(-1, 9)), f(self.light_quads, 9),
                            None if self.light_kinds is None else u(self.light_kinds),
                            len(self.box_mat), f(self.boxes, 18), u(self.box_mat),
                            None if self.mat_tex is None else u(self.mat_tex),
                            len(np.asarray(self.tex_type).reshape(-1)), u(self.tex_type), f(self.tex_params, 4),
                            u(self.tex_refs), len(np.asarray(self.perlin_vec).reshape(-1, 768)),
                            f(self.perlin_vec, 768), u(self.perlin_perm),
                            int(self.n_light_other), int(self.light_flags))
        return s, keep

    @staticmethod
    def from_c(s: "_capi.rtw_scene") -> "SceneSoA":
        def f(ptr, n, cols):
            return np.ctypeslib.as_array(ptr, shape=(n * cols,)).reshape(n, cols).copy() if n else np.zeros((0, cols))

        def u(ptr, n):
            return np.ctypeslib.as_array(ptr, shape=(n,)).copy() if n else np.zeros(0, np.uint32)

        return SceneSoA(f(s.spheres, s.n_spheres, 4), u(s.sphere_mat, s.n_spheres),
                        f(s.planes, s.n_planes, 6), u(s.plane_mat, s.n_planes),
                        u(s.mat_type, s.n_materials), f(s.mat_params, s.n_materials, 5),
                        f(s.lights, s.n_lights, 4), f(s.quads, s.n_quads, 9), u(s.quad_mat, s.n_quads),
                        f(s.light_quads, s.n_light_quads, 9),
                        u(s.light_kinds, s.n_lights + s.n_light_quads + s.n_light_other) if s.light_kinds else None,
                        f(s.boxes, s.n_boxes, 18), u(s.box_mat, s.n_boxes),
                        u(s.mat_tex, s.n_materials) if s.mat_tex else None,
                        u(s.tex_type, s.n_textures), f(s.tex_params, s.n_textures, 4),
                        u(s.tex_refs, 2 * s.n_textures).reshape(-1, 2),
                        f(s.perlin_vec, s.n_perlin, 768).reshape(-1, 256, 3),
                        u(s.perlin_perm, 768 * s.n_perlin).reshape(-1, 3, 256),
                        int(s.n_light_other), int(s.light_flags))


def flatten(world, lights) -> SceneSoA:
    """world: HittableList (or BoundedVolumeHierarchy) or SceneSoA; lights:
    a HittableList / BoundedVolumeHierarchy.  The light list's order is kept:
    it is the light pdf's sum order and the uniform pick's index.  Spheres
    and Quads sample themselves; Planes and Cuboids in a light list have the
    Hittable defaults (pdf 0, random (1, 0, 0); hittable.rs:175-181)."""
    if isinstance(world, SceneSoA):
        return world
    mats, mtypes, sph, smat, pl, pmat, qd, qmat = [], [], [], [], [], [], [], []
    textured = any(o.mat.texture is not None and o.mat.type in (RTW_LAMBERTIAN, RTW_DIFFUSE_LIGHT)
                   for o in world.objects)
    mtex, ttype, tpar, trefs, pvec, pperm = [], [], [], [], [], []
    tex_ids, perlin_ids = {}, {}

    def push_tex(t):
        if id(t) in tex_ids:
            return tex_ids[id(t)][0]
        k = len(ttype)
        tex_ids[id(t)] = (k, t)                       # keep t alive while its id() is a key
        if isinstance(t, SolidColour):
            ttype.append(RTW_TEX_SOLID)
            tpar.append(list(map(float, t.colour)) + [0.0])
            trefs.append([0, 0])
        elif isinstance(t, CheckerTexture):
            ttype.append(RTW_TEX_CHECKER)
            tpar.append([0.0, 0.0, 0.0, t.inv_scale])
            trefs.append([0, 0])
            trefs[k] = [push_tex(t.even), push_tex(t.odd)]
        else:
            ttype.append(RTW_TEX_NOISE)
            tpar.append([0.0, 0.0, 0.0, t.scale])
            if id(t.noise) not in perlin_ids:
                perlin_ids[id(t.noise)] = (len(pvec), t.noise)
                pvec.append(t.noise.rand_vec)
                pperm.append(t.noise.perm)
            trefs.append([perlin_ids[id(t.noise)][0], 0])
        return k

    def push(m: Material):
        mtypes.append(m.type)
        mats.append(list(m.albedo) + [m.fuzz, m.ior])
        if textured:
            if m.texture is not None and m.type in (RTW_LAMBERTIAN, RTW_DIFFUSE_LIGHT):
                mtex.append(push_tex(m.texture))
            else:
                mtex.append(push_tex(SolidColour(m.albedo)))
        return len(mtypes) - 1

    # materials numbered planes, spheres, quads, cuboids (as the C++ flatten)
    for o in world.objects:
        if isinstance(o, Plane):
            pl.append(list(o.point) + list(o.normal))
            pmat.append(push(o.mat))
    for o in world.objects:
        if isinstance(o, Sphere):
            sph.append(list(o.center) + [o.radius])
            smat.append(push(o.mat))
    for o in world.objects:
        if isinstance(o, Quad):
            qd.append(list(o.q) + list(o.u) + list(o.v))
            qmat.append(push(o.mat))
    bx, bmat = [], []
    for o in world.objects:
        if isinstance(o, Cuboid):
            bx.append(list(o.p) + list(o.q) + [v for row in o.xform.R for v in row] + list(o.xform.T))
            bmat.append(push(o.mat))
    li, lq, kinds = [], [], []
    for o in lights.objects:
        if isinstance(o, Sphere):
            li.append(list(o.center) + [o.radius])
            kinds.append(RTW_LIGHT_SPHERE)
        elif isinstance(o, Quad):
            lq.append(list(o.q) + list(o.u) + list(o.v))
            kinds.append(RTW_LIGHT_QUAD)
        else:
            kinds.append(RTW_LIGHT_DEFAULT)
    n_other = kinds.count(RTW_LIGHT_DEFAULT)
    flags = 0
    if isinstance(lights, BoundedVolumeHierarchy):
        if len(lights) > 5:
            raise RenderError(_capi.RTW_E_UNSUPPORTED, "a BVH light list of more than 5 entries (bvh.rs:78-92)")
        flags |= RTW_LIGHTS_BVH_LEAF
    return SceneSoA(np.array(sph, np.float64).reshape(-1, 4), np.array(smat, np.uint32),
                    np.array(pl, np.float64).reshape(-1, 6), np.array(pmat, np.uint32),
                    np.array(mtypes, np.uint32), np.array(mats, np.float64).reshape(-1, 5),
                    np.array(li, np.float64).reshape(-1, 4), np.array(qd, np.float64).reshape(-1, 9),
                    np.array(qmat, np.uint32), np.array(lq, np.float64).reshape(-1, 9),
                    np.array(kinds, np.uint32) if (lq or n_other) else None,
                    np.array(bx, np.float64).reshape(-1, 18), np.array(bmat, np.uint32),
                    np.array(mtex, np.uint32) if textured else None, np.array(ttype, np.uint32),
                    np.array(tpar, np.float64).reshape(-1, 4), np.array(trefs, np.uint32).reshape(-1, 2),
                    np.array(pvec, np.float64).reshape(-1, 256, 3), np.array(pperm, np.uint32).reshape(-1, 3, 256),
                    n_other, flags)


# ---------------------------------------------------------------- camera
class CameraBuilder:                          # camera.rs:28-112
    def __init__(self, raw: "_capi.rtw_camera_builder | None" = None):
        if raw is None:
            raw = _capi.rtw_camera_builder()
            _lib.rtw_camera_builder_default(C.byref(raw))
        self.raw = raw

    def _set3(self, name, v):
        getattr(self.raw, name)[:] = [float(x) for x in v]
        return self

    def with_aspect_ratio(self, v):
        self.raw.has_aspect_ratio, self.raw.aspect_ratio = 1, float(v)
        return self

    def with_image_width(self, v):
        self.raw.has_image_width, self.raw.image_width = 1, int(v)
        return self

    def with_image_height(self, v):
        self.raw.has_image_height, self.raw.image_height = 1, int(v)
        return self

    def with_samples_per_pixel(self, v):
        self.raw.samples_per_pixel = int(v)
        return self

    def with_max_depth(self, v):
        self.raw.max_depth = int(v)
        return self

    def with_background(self, c):
        return self._set3("background", c)

    def with_vfov(self, v):
        self.raw.vfov = float(v)
        return self

    def with_lookfrom(self, p):
        return self._set3("lookfrom", p)

    def with_lookat(self, p):
        return self._set3("lookat", p)

    def with_vup(self, v):
        return self._set3("vup", v)

    def with_defocus_angle(self, v):
        self.raw.defocus_angle = float(v)
        return self

    def with_focus_dist(self, v):
        self.raw.focus_dist = float(v)
        return self

    def build(self) -> "Camera":              # camera.rs:114-218
        cam = _capi.rtw_camera()
        rc = _lib.rtw_camera_build(C.byref(self.raw), C.byref(cam))
        if rc != 0:
            raise RenderError(rc, "CameraBuilder::build failed")
        return Camera(cam)

    def copy(self) -> "CameraBuilder":
        raw = _capi.rtw_camera_builder()
        C.pointer(raw)[0] = self.raw
        return CameraBuilder(raw)


class Camera:
    def __init__(self, raw: "_capi.rtw_camera"):
        self.raw = raw

    def __getattr__(self, name):
        raw = self.__dict__["raw"]
        v = getattr(raw, name)
        return tuple(v) if isinstance(v, C.Array) else v

    def render(self, world, lights, *, seed: int = 0x5EED0001, precision: int = RTW_F64,
               device: int = 0, devices=None, accel: int = RTW_ACCEL_AUTO) -> np.ndarray:
        """Camera::render (camera.rs:295-297) on the GPU: float64 sums [H, W, 3].
        The default is the parity mode (RTW_F64: the reference's f64 arithmetic,
        bit-identical to the oracle); precision=RTW_F32 opts into the faster
        speed mode, which agrees with the reference statistically.
        `devices` (a list of GPU indices) renders on all of them, one rank each
        (rtw_create_devices) -- the same image bit for bit."""
        with Renderer(device=device, precision=precision, devices=devices) as r:
            r.set_accel(accel)
            r.set_scene(flatten(world, lights))
            return r.render(self, seed)

    render_debug = render                     # camera.rs:299-312 (no sequential mode on a GPU)


class Renderer:
    """An rtw_ctx: a device (or, with `devices`, one rank per listed GPU:
    rtw_create_devices), a precision, a resident scene and work buffers."""

    def __init__(self, device: int = 0, precision: int = RTW_F32, *, devices=None, virtual_ranks=None):
        self.ctx = None
        if virtual_ranks is not None:
            # test mode (rtw_create_virtual): `virtual_ranks` ranks on `device`,
            # the gather by device copies -- the n-rank path on one GPU
            out = C.c_void_p()
            rc = _lib.rtw_create_virtual(device, int(virtual_ranks), precision, C.byref(out))
            if rc != 0:
                raise RenderError(rc, f"rtw_create_virtual({device}, {virtual_ranks}) failed (code {rc})")
            self.ctx = out.value
        elif devices is not None:
            devs = [int(d) for d in devices]
            arr = (C.c_int * max(len(devs), 1))(*devs)
            out = C.c_void_p()
            rc = _lib.rtw_create_devices(arr, len(devs), precision, C.byref(out))
            if rc != 0:
                raise RenderError(rc, f"rtw_create_devices({devs}) failed (code {rc}): an empty, repeated "
                                  "or not visible device, or a HIP / RCCL failure")
            self.ctx = out.value
            device = devs[0]
        else:
            self.ctx = _lib.rtw_create(device, precision)
            if not self.ctx:
                raise RenderError(_capi.RTW_E_DEVICE, f"rtw_create(device={device}) failed: no gfx950 "
                                  "device visible (this library has no CPU path)")
        self.device = device
        self.precision = precision
        self.stats = _capi.rtw_stats()

    @property
    def n_devices(self) -> int:
        return int(_lib.rtw_device_count(self.ctx))

    def rank_view(self, k: int) -> "_RankView":
        """Rank k's per-device context (stats / timings / last kernel)."""
        sub = _lib.rtw_device_ctx(self.ctx, k)
        if not sub:
            raise RenderError(_capi.RTW_E_INVALID, f"no rank {k}")
        return _RankView(self, k, sub, int(_lib.rtw_device_of(sub)), self.precision)

    def close(self):
        if self.ctx:
            _lib.rtw_destroy(self.ctx)
            self.ctx = None

    __del__ = close

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def _check(self, rc, what):
        if rc != 0:
            raise RenderError(rc, f"{what}: {_lib.rtw_last_error(self.ctx).decode()}")

    def set_chunk(self, chunk: int):
        self._check(_lib.rtw_set_chunk(self.ctx, chunk), "rtw_set_chunk")

    def set_tuning(self, key: str, value: int):
        self._check(_lib.rtw_set_tuning(self.ctx, key.encode(), int(value)), "rtw_set_tuning")

    def set_accel(self, accel: int):
        self._check(_lib.rtw_set_accel(self.ctx, accel), "rtw_set_accel")

    def set_scene(self, scene: SceneSoA):
        s, keep = scene.as_c()
        self._check(_lib.rtw_set_scene(self.ctx, C.byref(s)), "rtw_set_scene")
        del keep

    def render(self, cam: Camera, seed: int) -> np.ndarray:
        H, W = cam.raw.image_height, cam.raw.image_width
        out = np.zeros((H, W, 3), np.float64)
        self._check(_lib.rtw_render(self.ctx, C.byref(cam.raw), None, C.c_uint64(seed),
                                    out.ctypes.data_as(_capi._f64p), C.byref(self.stats)),
                    "rtw_render")
        return out

    def render_device(self, cam: Camera, seed: int, out_ptr: int, out_bytes: int, *,
                      rank: int = 0, nranks: int = 1, stream: int | None = None):
        """Asynchronous render of this rank's 8x8 tiles (T = rank mod nranks),
        packed, into device memory (rtw_render_device).  `stream` defaults to
        torch's current stream, so that the render is ordered after the torch
        work that prepared `out_ptr` and before the work that reads it."""
        if stream is None:
            stream = _torch_stream(self.device)
        self._check(_lib.rtw_render_device(self.ctx, C.byref(cam.raw), C.c_uint64(seed), rank,
                                           nranks, C.c_void_p(out_ptr) if out_ptr else None, out_bytes,
                                           C.c_void_p(stream) if stream else None),
                    "rtw_render_device")

    def render_image_device(self, cam: Camera, seed: int, image_ptr: int, image_bytes: int, *,
                            stream: int | None = None):
        """Asynchronous render of the whole image [H, W, 3] into device memory
        of the first device (rtw_render_image_device): every device of the
        context renders its share, one RCCL gather, the assembly on `stream`
        (torch's current stream of the first device by default)."""
        if stream is None:
            stream = _torch_stream(self.device)
        self._check(_lib.rtw_render_image_device(self.ctx, C.byref(cam.raw), C.c_uint64(seed),
                                                 C.c_void_p(image_ptr) if image_ptr else None, image_bytes,
                                                 C.c_void_p(stream) if stream else None),
                    "rtw_render_image_device")

    def assemble_tiles(self, ranks_ptr: int, rank_stride_bytes: int, nranks: int, width: int,
                       height: int, image_ptr: int, *, stream: int | None = None):
        """The ranks' gathered packed tiles -> the image [H, W, 3] on the device
        (rtw_assemble_tiles), on torch's current stream by default."""
        if stream is None:
            stream = _torch_stream(self.device)
        self._check(_lib.rtw_assemble_tiles(self.ctx, C.c_void_p(ranks_ptr), rank_stride_bytes, nranks,
                                            width, height, C.c_void_p(image_ptr),
                                            C.c_void_p(stream) if stream else None),
                    "rtw_assemble_tiles")

    def set_split(self, width: int, height: int, nranks: int, tile_rank=None, tile_cost=None):
        """Renders and assemblies of a width x height image over nranks ranks
        follow this tile -> rank split from now on (rtw_set_split, ABI 10);
        None restores the round robin.  tile_cost orders each rank's tasks."""
        n = n_tiles(width, height)

        def arr(a):
            if a is None:
                return None, None
            a = np.ascontiguousarray(np.asarray(a, np.uint32).reshape(-1))
            if a.size != n:
                raise RenderError(_capi.RTW_E_INVALID, f"split arrays need {n} entries, got {a.size}")
            return a, a.ctypes.data_as(_capi._u32p)
        r, rp = arr(tile_rank)
        c, cp = arr(tile_cost)
        self._check(_lib.rtw_set_split(self.ctx, width, height, nranks, rp, cp), "rtw_set_split")

    def get_split(self, width: int, height: int, nranks: int):
        """(kind, tile_rank) of the split renders of this size and rank count
        follow (rtw_get_split): kind 0 = the round robin (tile_rank None),
        1 = set by set_split, 2 = dealt by the context itself (balance)."""
        out = np.zeros(n_tiles(width, height), np.uint32)
        kind = _lib.rtw_get_split(self.ctx, width, height, nranks, out.ctypes.data_as(_capi._u32p))
        if kind < 0:
            self._check(kind, "rtw_get_split")
        return int(kind), (out if kind else None)

    def tile_costs(self, cam: Camera, rank: int = 0, nranks: int = 1, out=None) -> np.ndarray:
        """The tile costs this context counted in its first render of (cam,
        rank, nranks) (rtw_tile_costs): uint32 [n_tiles], the rank's tiles
        filled in (zeros elsewhere, or `out`'s entries kept).  Waits."""
        n = n_tiles(cam.image_width, cam.image_height)
        out = np.zeros(n, np.uint32) if out is None else out
        if out.dtype != np.uint32 or out.size != n or not out.flags.c_contiguous:
            raise RenderError(_capi.RTW_E_INVALID, "out must be a contiguous uint32 array of n_tiles")
        self._check(_lib.rtw_tile_costs(self.ctx, C.byref(cam.raw), rank, nranks, out.ctypes.data_as(_capi._u32p)),
                    "rtw_tile_costs")
        return out

    def get_timings(self, n: int = 64):
        """(render_ms, total_ms) lists for the last n renders (HIP events)."""
        a, b = (C.c_float * n)(), (C.c_float * n)()
        got = _lib.rtw_get_timings(self.ctx, a, b, n)
        if got < 0:
            self._check(got, "rtw_get_timings")
        return list(a[:got]), list(b[:got])

    def last_kernel(self):
        """(kernel, options) of the render kernel the last render launched
        (rtw_last_kernel), or None before any: render_kernel<R, kernel, options>."""
        v = _lib.rtw_last_kernel(self.ctx)
        if v < 0:
            self._check(v, "rtw_last_kernel")
        return None if v == 0 else (v >> 8, v & 0xff)

    def get_stats(self) -> "_capi.rtw_stats":
        self._check(_lib.rtw_get_stats(self.ctx, C.byref(self.stats)), "rtw_get_stats")
        return self.stats


class _RankView(Renderer):
    """One rank of a multi-device Renderer (not owned: close() is a no-op).
    It keeps its parent alive and refuses to run once the parent is closed
    (the rank's context is freed with it)."""

    def __init__(self, parent, k, ctx, device, precision):   # noqa: D107  (no rtw_create)
        self._parent = parent
        self._k = k
        self._sub = ctx
        self.device = device
        self.precision = precision
        self.stats = _capi.rtw_stats()

    @property
    def ctx(self):
        if self._parent is None or not self._parent.ctx:
            raise RenderError(_capi.RTW_E_INVALID, "rank view of a closed Renderer")
        return self._sub

    def get_stats(self) -> "_capi.rtw_stats":
        """This rank's own counters (rtw_get_stats_rank; rank 0 too)."""
        self.ctx
        self._check(_lib.rtw_get_stats_rank(self._parent.ctx, self._k, C.byref(self.stats)), "rtw_get_stats_rank")
        return self.stats

    def close(self):
        self._parent = None

    __del__ = close


def tiles_for_rank(width: int, height: int, rank: int, nranks: int) -> int:
    """8x8 tiles rank `rank` of `nranks` renders (rtw_tiles_for_rank)."""
    return int(_lib.rtw_tiles_for_rank(width, height, rank, nranks))


def tile_size() -> int:
    return int(_lib.rtw_tile_size())


def n_tiles(width: int, height: int) -> int:
    t = tile_size()
    return ((width + t - 1) // t) * ((height + t - 1) // t)


def split_deal(tile_cost, width: int, height: int, nranks: int) -> np.ndarray:
    """The tiles dealt to nranks ranks by cost (rtw_split_deal): uint32
    tile -> rank, each rank keeping its round-robin tile count."""
    n = n_tiles(width, height)
    cost = np.ascontiguousarray(np.asarray(tile_cost, np.uint32).reshape(-1))
    if cost.size != n:
        raise RenderError(_capi.RTW_E_INVALID, f"tile_cost needs {n} entries, got {cost.size}")
    out = np.zeros(n, np.uint32)
    rc = _lib.rtw_split_deal(cost.ctypes.data_as(_capi._u32p), width, height, nranks, out.ctypes.data_as(_capi._u32p))
    if rc != 0:
        raise RenderError(rc, "rtw_split_deal failed")
    return out


RTW_STREAM_NULL = 1   # include/rtw.h: the device's null (legacy default) stream


def torch_stream(device: int) -> int:
    """The rtw stream argument for torch's current stream on `device` (the
    Renderer's device, whatever torch's current device is): its hipStream_t,
    or RTW_STREAM_NULL when that is torch's default stream (handle 0, the
    device's null stream -- passing 0 would mean the context's own,
    unordered stream); 0 -- the context's own stream -- when torch has no GPU."""
    try:
        import torch
        if torch.cuda.is_available():
            h = int(torch.cuda.current_stream(device).cuda_stream)
            return h if h else RTW_STREAM_NULL
    except ImportError:
        pass
    return 0


_torch_stream = torch_stream


# ---------------------------------------------------------------- scenes
class scenes:                                 # scenes/src/lib.rs
    @staticmethod
    def simple_soa(seed: int = 0x5EED0001, n: int = 11):
        """(SceneSoA, CameraBuilder) straight from the C++ generator."""
        w = _lib.rtw_scene_simple(C.c_uint64(seed & 0xFFFFFFFFFFFFFFFF), n)
        if not w:
            raise RenderError(_capi.RTW_E_INVALID, "rtw_scene_simple failed")
        try:
            soa = SceneSoA.from_c(_lib.rtw_world_scene(w).contents)
            b = _capi.rtw_camera_builder()
            _lib.rtw_world_camera_builder(w, C.byref(b))
        finally:
            _lib.rtw_world_free(w)
        return soa, CameraBuilder(b)

    NAMES = ("cornell_box", "debug", "checkered_spheres", "perlin_spheres", "plane", "simple",
             "simple_light", "simple_transform")      # bin/src/main.rs:29-38

    @staticmethod
    def named_soa(name: str, seed: int = 0x5EED0001):
        """(SceneSoA, CameraBuilder) of a reference scene by its main.rs name
        (scenes.NAMES); `seed` drives simple's generator and the Perlin tables."""
        w = _lib.rtw_scene_named(name.encode(), C.c_uint64(seed & 0xFFFFFFFFFFFFFFFF))
        if not w:
            raise RenderError(_capi.RTW_E_UNSUPPORTED, f"scene {name!r} is not in this build")
        try:
            soa = SceneSoA.from_c(_lib.rtw_world_scene(w).contents)
            b = _capi.rtw_camera_builder()
            _lib.rtw_world_camera_builder(w, C.byref(b))
        finally:
            _lib.rtw_world_free(w)
        return soa, CameraBuilder(b)

    @staticmethod
    def cornell_box_soa():
        return scenes.named_soa("cornell_box")

    @staticmethod
    def simple(seed: int = 0x5EED0001, n: int = 11):
        """scenes::simple -> (world, lights, CameraBuilder) as object lists."""
        soa, builder = scenes.simple_soa(seed, n)
        world, lights = HittableList(), HittableList()
        for pl, m in zip(soa.planes, soa.plane_mat):
            world.add(Plane(tuple(pl[:3]), tuple(pl[3:]), _mat(soa, m)))
        for sp, m in zip(soa.spheres, soa.sphere_mat):
            world.add(Sphere(tuple(sp[:3]), float(sp[3]), _mat(soa, m)))
        for li in soa.lights:
            lights.add(Sphere(tuple(li[:3]), float(li[3]), INVISIBLE))
        return world, lights, builder


def _mat(soa, m):
    p = soa.mat_params[m]
    return Material(int(soa.mat_type[m]), (float(p[0]), float(p[1]), float(p[2])), float(p[3]),
                    float(p[4]))


# ---------------------------------------------------------------- output
def _sums(sums: np.ndarray):
    """(contiguous array, ctypes pointer, f32?) of float32 or float64 sums."""
    if np.asarray(sums).dtype == np.float32:
        s = np.ascontiguousarray(sums, np.float32)
        return s, s.ctypes.data_as(_capi._f32p), True
    s = np.ascontiguousarray(sums, np.float64)
    return s, s.ctypes.data_as(_capi._f64p), False


def encode_rgb8(sums: np.ndarray, spp: int) -> np.ndarray:
    """SampledColour Display (colour.rs:14-36), rows flipped top-first: uint8 [H, W, 3].
    float32 sums (a speed-mode render) are widened to f64 exactly first."""
    s, ptr, f32 = _sums(sums)
    H, W = s.shape[:2]
    out = np.zeros((H, W, 3), np.uint8)
    fn = _lib.rtw_encode_rgb8_f32 if f32 else _lib.rtw_encode_rgb8
    fn(ptr, W, H, spp, out.ctypes.data_as(C.POINTER(C.c_uint8)))
    return out


def write_ppm(path: str, sums: np.ndarray, spp: int) -> int:
    """The reference's P3 image.ppm (bin/src/main.rs:89-104)."""
    s, ptr, f32 = _sums(sums)
    H, W = s.shape[:2]
    n = (_lib.rtw_write_ppm_f32 if f32 else _lib.rtw_write_ppm)(path.encode(), ptr, W, H, spp)
    if n < 0:
        raise RenderError(n, f"cannot write {path}")
    return n
