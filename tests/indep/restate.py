"""Independent scalar restatement of the reference's per-sample integrator --
TEST INFRASTRUCTURE ONLY (a checker of the checker: never on the product path).

Written straight from the Rust sources of N9199/ray_tracing_weekend (paths
relative to the reference root), NOT from oracle/rtw_oracle.c, so that the
oracle's reading of the Rust is checked by a second, separate reading:

  Camera::get_ray                   shared/src/camera.rs:274-293
  ray_colour_tail_call              shared/src/camera.rs:459-522
  Sphere::hit / pdf_value / random  shared/src/entities/sphere.rs:61-127
  Plane::hit / get_aabbox           shared/src/entities/plane.rs:24-113
  Quad::new / hit / pdf / random    shared/src/entities/quadrilateral.rs:29-118
  Cuboid::new / hit                 shared/src/entities/cuboid.rs:24-58
  Transformed<T>::hit               shared/src/entities/transformations.rs:14-29
  Transformation / Matrix3          geometry/src/transformations.rs:84-125, geometry/src/matrix3.rs:8-84
  AABBox (from_points, pad, hit)    geometry/src/aabox.rs:150-226, shared/src/hittable.rs:38-86
  bounded_hit / list hit (min_by)   shared/src/hittable.rs:190-211, hittable_list.rs:394-420
  HitRecord::new                    shared/src/hittable.rs:100-126
  Lambertian / Metal / Dialectric   shared/src/material.rs:357-488
  DiffuseLight::emitted             shared/src/material.rs:508-514
  Cosine / Hittable / Mixture pdf   shared/src/pdf.rs:33-101
  Onb                               geometry/src/onb.rs:8-35
  UnitSphere / UnitDisk / cosine    shared/src/utils.rs:99-161
  Vec3 ops (dot order, reflect, refract, Sum)   geometry/src/vec3/vec.rs
  CheckerTexture / SolidColour      shared/src/texture.rs:15-55
  BVH leaf light list pdf           shared/src/hittable_collections/bvh.rs:67-76, 191-194

Python floats are IEEE binary64 with correctly rounded + - * / and sqrt, so
every expression below rounds exactly like the Rust f64 code it restates, in
the same operation order (Rust never contracts a*b+c into an FMA).

Where the reference is not reproducible the build's documented conventions
(DESIGN.md §2 "Deliberate differences") are restated from their published
algorithms, not from the oracle's code:
  * RNG: thread_rng-seeded SmallRng per pixel is unobtainable; every (pixel,
    sample) gets xoshiro256++ seeded through splitmix64 (Vigna's published
    generators) from (seed, pixel, sample).  rand 0.8.6's Standard / Open01 /
    Uniform::new_inclusive / gen_range(u32) sit on top of it.
  * The light pick is ONE gen_index(n) draw (choose()'s reservoir step would
    add a gen_index(1) and rotate the index; same uniform law), UnitSphere does
    not shuffle its i.i.d. coordinates.
  * cos / sin of 2*pi*r: fdlibm's published __kernel_sin / __kernel_cos
    polynomials after the exact quadrant reduction of r.
  * The reference's HittableList iterates its objects grouped by TypeId (an
    order rustc picks); the build's order is planes, quads, cuboids, spheres,
    and the light list in the given order.  Only exact ties of t depend on it.
"""
from __future__ import annotations

import math

EPS = 2.220446049250313e-16          # f64::EPSILON
INF = float("inf")
PI = math.pi
M64 = (1 << 64) - 1

LAMBERTIAN, METAL, DIELECTRIC, INVISIBLE, DIFFUSE_LIGHT = 0, 1, 2, 3, 4
TEX_SOLID, TEX_CHECKER = 0, 1
LIGHT_SPHERE, LIGHT_QUAD, LIGHT_DEFAULT = 0, 1, 2


# --------------------------------------------------------------- Vec3 (vec.rs)
def add(a, b):
    return (a[0] + b[0], a[1] + b[1], a[2] + b[2])


def sub(a, b):
    return (a[0] - b[0], a[1] - b[1], a[2] - b[2])


def neg(a):
    return (-a[0], -a[1], -a[2])


def muls(a, s):
    return (a[0] * s, a[1] * s, a[2] * s)


def mulv(a, b):
    return (a[0] * b[0], a[1] * b[1], a[2] * b[2])


def fdiv(a, b):                      # IEEE a / b (Python raises on b == 0)
    try:
        return a / b
    except ZeroDivisionError:
        if a != a or a == 0.0:
            return float("nan")
        return math.copysign(INF, a) * math.copysign(1.0, b)


def divs(a, s):
    return (fdiv(a[0], s), fdiv(a[1], s), fdiv(a[2], s))


def dot(a, b):                       # self.x * rhs.x + self.y * rhs.y + self.z * rhs.z
    return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]


def cross(a, b):
    return (a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0])


def length(a):
    return math.sqrt(dot(a, a))


def normalize(a):                    # self / self.length()
    return divs(a, length(a))


def reflect(v, n):                   # self - other * 2. * self.dot(other)
    return sub(v, muls(muls(n, 2.0), dot(v, n)))


def refract(v, n, eta):
    cos_theta = fmin(dot(v, neg(n)), 1.0)
    perp = muls(add(v, muls(n, cos_theta)), eta)
    par = muls(n, -math.sqrt(1.0 - dot(perp, perp)))
    return add(perp, par)


def fmin(a, b):                      # f64::min: NaN-ignoring
    if a != a:
        return b
    if b != b:
        return a
    return a if a < b else b


def fmax(a, b):
    if a != a:
        return b
    if b != b:
        return a
    return a if a > b else b


def sqrt(x):                         # f64::sqrt: NaN for x < 0
    return math.sqrt(x) if x >= 0 else (x if x != x else float("nan"))


# ------------------------------------------------------------- RNG (see header)
def _mix64(z):
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def _rotl(x, k):
    return ((x << k) | (x >> (64 - k))) & M64


class Rng:
    """xoshiro256++ (Blackman & Vigna) seeded by a splitmix64 stream."""

    def __init__(self, seed, pixel, sample):
        k = _mix64((seed + 0x9E3779B97F4A7C15 * (pixel + 1)) & M64)
        k = _mix64(k ^ ((0xD1B54A32D192ED03 * (sample + 1)) & M64))
        self.s = []
        for _ in range(4):
            k = (k + 0x9E3779B97F4A7C15) & M64
            self.s.append(_mix64(k))

    def next_u64(self):
        s = self.s
        result = (_rotl((s[0] + s[3]) & M64, 23) + s[0]) & M64
        t = (s[1] << 17) & M64
        s[2] ^= s[0]
        s[3] ^= s[1]
        s[1] ^= s[2]
        s[0] ^= s[3]
        s[2] ^= t
        s[3] = _rotl(s[3], 45)
        return result

    def standard(self):              # rand 0.8.6 Standard for f64: (v >> 11) * 2^-53
        return (self.next_u64() >> 11) * (1.0 / 9007199254740992.0)

    def _one_two(self):              # (v >> 12) with exponent 0: [1, 2)
        return 1.0 + (self.next_u64() >> 12) * 2.0 ** -52

    def open01(self):                # Open01: [1, 2) - (1 - EPSILON / 2)
        return self._one_two() - (1.0 - EPS / 2.0)

    def uniform(self, low, scale):   # UniformFloat::sample: value0_1 * scale + low
        return (self._one_two() - 1.0) * scale + low

    def gen_index(self, n):          # gen_range(0..n) on u32: widening multiply + zone
        zone = ((n << (32 - n.bit_length())) & 0xFFFFFFFF) - 1
        while True:
            v = self.next_u64() >> 32
            m = v * n
            if (m & 0xFFFFFFFF) <= zone:
                return m >> 32


def uniform_inclusive_scale(low, high):
    """Uniform::new_inclusive (rand 0.8.6 UniformFloat): scale = (high - low) /
    max_rand, lowered ulp by ulp until scale * max_rand + low <= high."""
    max_rand = 1.0 - 2.0 ** -52
    scale = (high - low) / max_rand
    while scale * max_rand + low > high:
        scale = math.nextafter(scale, 0.0)
    return scale


# fdlibm __kernel_sin / __kernel_cos (s_sin.c / k_cos.c constants)
_S = (-1.66666666666666324348e-01, 8.33333333332248946124e-03, -1.98412698298579493134e-04,
      2.75573137070700676789e-06, -2.50507602534068634195e-08, 1.58969099521155010221e-10)
_C = (4.16666666666666019037e-02, -1.38888888888741095749e-03, 2.48015872894767294178e-05,
      -2.75573143513906633035e-07, 2.08757232129817482790e-09, -1.13596475577881948265e-11)


def _k_sin(x):
    z = x * x
    v = z * x
    r = _S[1] + z * (_S[2] + z * (_S[3] + z * (_S[4] + z * _S[5])))
    return x + v * (_S[0] + z * r)


def _k_cos(x):
    import struct
    z = x * x
    r = z * (_C[0] + z * (_C[1] + z * (_C[2] + z * (_C[3] + z * (_C[4] + z * _C[5])))))
    ax = abs(x)
    if ax < 0.3:
        return 1.0 - (0.5 * z - z * r)
    if ax > 0.78125:
        qx = 0.28125
    else:                            # ax / 4 truncated to its high word
        b = struct.unpack("<Q", struct.pack("<d", ax))[0]
        b = (b - 0x0020000000000000) & 0xFFFFFFFF00000000
        qx = struct.unpack("<d", struct.pack("<Q", b))[0]
    hz = 0.5 * z - qx
    return (1.0 - qx) - (hz - z * r)


def sincos_2pi(r):
    """(sin, cos) of 2 pi r: r = q/4 + f exactly, then the kernels on 2 pi f."""
    q = float(round(r * 4.0))        # round half to even, like rint
    f = r - q * 0.25
    x = f * (2.0 * PI)
    ks, kc = _k_sin(x), _k_cos(x)
    return [(ks, kc), (kc, -ks), (-ks, -kc), (-kc, ks)][int(q) & 3]


# ------------------------------------------------------------ samplers (utils.rs)
def unit_sphere(g):
    while True:
        out = (2.0 * g.standard() - 1.0, 2.0 * g.standard() - 1.0, 2.0 * g.standard() - 1.0)
        if dot(out, out) < 1.0:
            return out


def unit_disk(g):
    while True:
        x = 2.0 * g.standard() - 1.0
        z = 2.0 * g.standard() - 1.0
        out = (x, 0.0, z)
        if dot(out, out) < 1.0:
            return out


def cosine_hemisphere(g):
    r1 = g.standard()
    r2 = g.standard()
    s, c = sincos_2pi(r1)            # phi = 2 PI r1
    return (c * math.sqrt(r2), s * math.sqrt(r2), math.sqrt(1.0 - r2))


class Onb:                           # onb.rs:8-35
    def __init__(self, n):
        w = normalize(n)
        a = (0.0, 1.0, 0.0) if abs(w[0]) > 0.9 else (1.0, 0.0, 0.0)
        v = normalize(cross(w, a))
        self.u, self.v, self.w = cross(w, v), v, w

    def transform(self, x):          # (0..3).map(|i| e[i] * x[i]).sum(): fold from zero
        acc = (0.0, 0.0, 0.0)
        acc = add(acc, muls(self.u, x[0]))
        acc = add(acc, muls(self.v, x[1]))
        return add(acc, muls(self.w, x[2]))


# ------------------------------------------------------------------ AABBox
class AABB:
    def __init__(self, lo, hi):
        self.lo, self.hi = tuple(lo), tuple(hi)

    @staticmethod
    def from_points(pts):            # first point, then enclose (pad_to_minimum each time)
        b = AABB(pts[0], pts[0])
        for p in pts[1:]:
            b = b.enclose(AABB(p, p))
        return b

    def enclose(self, o):
        lo = [fmin(a, b) for a, b in zip(self.lo, o.lo)]
        hi = [fmax(a, b) for a, b in zip(self.hi, o.hi)]
        for k in range(3):           # pad_to_minimum, DELTA = 0.0001
            if hi[k] - lo[k] < 0.0001:
                lo[k] -= 0.0001
                hi[k] += 0.0001
        return AABB(lo, hi)

    def points(self):                # get_points order
        (a, b, c), (d, e, f) = self.lo, self.hi
        return [(a, b, c), (a, e, c), (a, b, f), (a, e, f), (d, b, c), (d, e, c), (d, b, f), (d, e, f)]

    def is_hit(self, o, d, tmin_r, tmax_r):   # AABoxHit::hit, hittable.rs:39-86
        def slab(k):
            t0 = (self.lo[k] - o[k]) / d[k] if d[k] != 0 else _div0(self.lo[k] - o[k], d[k])
            t1 = (self.hi[k] - o[k]) / d[k] if d[k] != 0 else _div0(self.hi[k] - o[k], d[k])
            return (t1, t0) if math.copysign(1.0, d[k]) < 0 else (t0, t1)
        tmin, tmax = slab(0)
        y0, y1 = slab(1)
        if tmax < y0 or tmin > y1:
            return False
        tmin, tmax = fmax(tmin, y0), fmin(tmax, y1)
        z0, z1 = slab(2)
        if tmax < z0 or tmin > z1:
            return False
        tmin, tmax = fmax(tmin, z0), fmin(tmax, z1)
        return fmax(tmin_r, tmin) <= fmin(tmax_r, tmax)


def _div0(a, b):                     # IEEE a / +-0
    if a != a or a == 0:
        return float("nan")
    return math.copysign(INF, a) * math.copysign(1.0, b)


# ---------------------------------------------------------------- geometry
class Hit:
    """HitRecord::new (hittable.rs:100-126)."""

    def __init__(self, o, d, t, outward, u, v, mat, p=None):
        self.t = t
        self.p = add(o, muls(d, t)) if p is None else p      # r.at(t) = origin + direction * t
        self.front = dot(d, outward) < 0.0
        self.normal = outward if self.front else neg(outward)
        self.u, self.v, self.mat = u, v, mat


class Sphere:
    def __init__(self, c, r, mat):
        self.c, self.r, self.mat = tuple(c), r, mat
        self.aabb = AABB(sub(self.c, (r, r, r)), add(self.c, (r, r, r)))

    def hit(self, o, d, lo, hi):
        oc = sub(o, self.c)
        a = dot(d, d)
        half_b = dot(d, oc)
        c = dot(oc, oc) - self.r * self.r
        disc = half_b * half_b - a * c
        if not disc > 0.0:
            return None
        sq = math.sqrt(disc)
        root = fdiv(-half_b - sq, a)
        if not (lo <= root <= hi):
            root = fdiv(-half_b + sq, a)
            if not (lo <= root <= hi):
                return None
        p = add(o, muls(d, root))
        outward = divs(sub(p, self.c), self.r)
        u = fdiv(math.atan2(-outward[2], outward[0]), 2.0 * PI)   # get_sphere_uv
        v = math.acos(outward[1]) / PI if -1.0 <= outward[1] <= 1.0 else float("nan")
        return Hit(o, d, root, outward, u, v, self.mat, p)

    def pdf_value(self, o, d):
        if self.hit(o, d, 0.0, INF) is None:
            return 0.0
        dist2 = dot(sub(self.c, o), sub(self.c, o))
        cos_theta_max = sqrt(1.0 - fdiv(self.r * self.r, dist2))
        return fdiv(1.0, 2.0 * PI * (1.0 - cos_theta_max))

    def random(self, o, g):
        direction = sub(self.c, o)
        distance = length(direction)
        uvw = Onb(direction)
        r1 = g.standard()
        r2 = g.standard()
        z = 1.0 + r1 * (sqrt(1.0 - fdiv(self.r * self.r, distance * distance)) - 1.0)
        s, c = sincos_2pi(r2)        # phi = 2 PI r2
        return uvw.transform((c * sqrt(1.0 - z * z), s * sqrt(1.0 - z * z), z))


class Plane:
    def __init__(self, p, n, mat):
        self.p, self.n, self.mat = tuple(p), normalize(tuple(n)), mat
        n = self.n
        pin = [abs(n[(k + 1) % 3]) < EPS and abs(n[(k + 2) % 3]) < EPS for k in range(3)]
        self.aabb = AABB([0.0 if f else -INF for f in pin], [0.0 if f else INF for f in pin])
        self.panics = 0

    def uv(self, pnt):               # get_plane_uv, plane.rs:40-54
        V = (0.0, 1.0, 0.0)
        theta = math.atan2(length(cross(self.n, V)), dot(self.n, V))
        if theta <= EPS:
            return pnt[0], pnt[2]
        k = normalize(cross(self.n, V))
        vec = sub(pnt, self.p)
        rot = add(add(muls(vec, math.cos(theta)), muls(cross(k, vec), math.sin(theta))),
                  muls(muls(k, dot(k, vec)), 1.0 - math.cos(theta)))
        return _fract(rot[0]), _fract(rot[2])

    def hit(self, o, d, lo, hi):
        denom = dot(d, self.n)
        if not denom > EPS:
            return None
        t = -fdiv(dot(sub(o, self.p), self.n), denom)
        pnt = add(o, muls(d, t))
        u, v = self.uv(pnt)
        if not (math.isfinite(u) and math.isfinite(v)):
            self.panics += 1         # plane.rs:67-69 panics
        if not (lo <= t <= hi):
            return None
        return Hit(o, d, t, self.n, u, v, self.mat)


class Quad:
    def __init__(self, q, u, v, mat):
        self.q, self.u, self.v, self.mat = tuple(q), tuple(u), tuple(v), mat
        q, u, v = self.q, self.u, self.v
        self.aabb = AABB.from_points([add(q, muls(add(u, v), 0.5)), q, add(q, v), add(q, u), add(add(q, u), v)])
        normal = cross(u, v)
        self.w = divs(normal, dot(normal, normal))
        self.area = length(normal)
        self.n = divs(normal, self.area)

    def hit(self, o, d, lo, hi):
        denom = dot(d, self.n)
        if not abs(denom) > EPS:
            return None
        t = -fdiv(dot(sub(o, self.q), self.n), denom)
        if not (lo <= t <= hi):
            return None
        pnt = add(o, muls(d, t))
        pq = sub(pnt, self.q)
        a = dot(cross(pq, self.v), self.w)
        b = dot(cross(self.u, pq), self.w)
        if not (0.0 <= a <= 1.0 and 0.0 <= b <= 1.0):
            return None
        return Hit(o, d, t, self.n, a, b, self.mat, pnt)

    def pdf_value(self, o, d):
        rec = self.hit(o, d, 0.0, INF)
        if rec is None:
            return 0.0
        distance_squared = rec.t * rec.t * dot(d, d)
        cosine = abs(fdiv(dot(d, rec.normal), length(d)))
        return fdiv(distance_squared, cosine * self.area)

    def random(self, o, g):
        p = add(add(self.q, muls(self.u, g.open01())), muls(self.v, g.open01()))
        return sub(p, o)


def _mat_vec(M, v):                  # Mul<Vec3> for Matrix3: row . v
    return (dot(M[0], v), dot(M[1], v), dot(M[2], v))


def _inverse(R, T):                  # Transformation::inverse via Matrix3::inverse
    (a, b, c), (d, e, f), (g, h, i) = R
    det = a * (e * i - f * h) + b * (f * g - d * i) + c * (d * h - e * g)
    if not (math.isfinite(det) and det != 0.0 and abs(det) >= 2.2250738585072014e-308):
        return None
    ca, cb, cc = e * i - f * h, f * g - d * i, d * h - e * g
    cd, ce, cf = c * h - b * i, a * i - c * g, b * g - a * h
    cg, ch, ci = b * f - c * e, c * d - a * f, a * e - b * d
    Ri = ((ca / det, cd / det, cg / det), (cb / det, ce / det, ch / det), (cc / det, cf / det, ci / det))
    return Ri, neg(_mat_vec(Ri, T))


class TransformedCuboid:
    def __init__(self, p, q, R, T, mat):
        self.mat = mat
        box = AABB.from_points([tuple(p), tuple(q)])
        mn, mx = box.lo, box.hi
        delta = sub(mx, mn)
        dx, dy, dz = (delta[0], 0.0, 0.0), (0.0, delta[1], 0.0), (0.0, 0.0, delta[2])
        self.quads = [Quad(mn, dx, dy, mat), Quad(mn, dy, dz, mat), Quad(mn, dx, dz, mat),
                      Quad(mx, neg(dx), neg(dy), mat), Quad(mx, neg(dy), neg(dz), mat),
                      Quad(mx, neg(dx), neg(dz), mat)]
        self.R = tuple(tuple(r) for r in R)
        self.T = tuple(T)
        inner = self.quads[0].aabb
        for qd in self.quads[1:]:
            inner = inner.enclose(qd.aabb)
        self.aabb = AABB.from_points([add(_mat_vec(self.R, pt), self.T) for pt in inner.points()])
        self.inv = _inverse(self.R, self.T)

    def hit(self, o, d, lo, hi):
        if self.inv is None:
            return None
        Ri, Ti = self.inv
        o2 = add(_mat_vec(Ri, o), Ti)
        d2 = add(_mat_vec(Ri, d), Ti)          # transform_vector3d also translates
        best = None
        for qd in self.quads:                  # Cuboid::hit: quads without their boxes
            rec = qd.hit(o2, d2, lo, hi)
            if rec is not None and (best is None or rec.t < best.t):
                best = rec
        if best is not None:
            best.p = add(_mat_vec(self.R, best.p), self.T)
        return best


# ------------------------------------------------------------------- scene
class World:
    def __init__(self, soa):
        mt, mp = list(map(int, soa.mat_type)), [tuple(map(float, r)) for r in soa.mat_params]
        self.mat_type, self.mat_params = mt, mp
        self.mat_tex = None if soa.mat_tex is None else list(map(int, soa.mat_tex))
        self.tex = [(int(k), tuple(map(float, p)), tuple(map(int, r)))
                    for k, p, r in zip(soa.tex_type, soa.tex_params, soa.tex_refs)]
        self.objects = []
        self.objects += [Plane(p[:3], p[3:6], int(m)) for p, m in zip(soa.planes, soa.plane_mat)]
        self.objects += [Quad(q[:3], q[3:6], q[6:9], int(m)) for q, m in zip(soa.quads, soa.quad_mat)]
        self.objects += [TransformedCuboid(b[0:3], b[3:6], (b[6:9], b[9:12], b[12:15]), b[15:18], int(m))
                         for b, m in zip(soa.boxes, soa.box_mat)]
        self.objects += [Sphere(s[:3], float(s[3]), int(m)) for s, m in zip(soa.spheres, soa.sphere_mat)]
        kinds = soa.light_kinds
        if kinds is None:
            kinds = [LIGHT_SPHERE] * len(soa.lights)
        ns = nq = 0
        self.lights = []
        for k in map(int, kinds):
            if k == LIGHT_SPHERE:
                self.lights.append(Sphere(soa.lights[ns][:3], float(soa.lights[ns][3]), INVISIBLE))
                ns += 1
            elif k == LIGHT_QUAD:
                q = soa.light_quads[nq]
                self.lights.append(Quad(q[:3], q[3:6], q[6:9], INVISIBLE))
                nq += 1
            else:
                self.lights.append(None)           # Hittable defaults: pdf 0, random (1, 0, 0)
        self.bvh_leaf = bool(int(soa.light_flags) & 1)

    def hit(self, o, d):             # list hit: bounded_hit of every object, first minimum of t
        best = None
        for ob in self.objects:
            if not ob.aabb.is_hit(o, d, EPS, INF):
                continue
            rec = ob.hit(o, d, EPS, INF)
            if rec is not None and (best is None or rec.t < best.t):
                best = rec
        return best

    def lights_pdf(self, o, d):      # HittableList::pdf_value: fold from 0. / len
        acc = 0.0
        for L in self.lights:
            acc = acc + (0.0 if L is None else L.pdf_value(o, d))
        n = float(len(self.lights))
        p = fdiv(acc, n)
        if self.bvh_leaf:            # BVH leaf: list pdf * len, then / len
            p = fdiv(p * n, n)
        return p

    def lights_random(self, o, g):
        L = self.lights[g.gen_index(len(self.lights))]
        return (1.0, 0.0, 0.0) if L is None else L.random(o, g)

    def colour(self, m, u, v, p):    # Texture::get_colour for material m
        if self.mat_tex is None:
            return self.mat_params[m][:3]
        tid = self.mat_tex[m]
        while True:
            kind, tp, refs = self.tex[tid]
            if kind == TEX_CHECKER:
                s = _floor(u * tp[3]) + _floor(v * tp[3])
                tid = refs[0] if math.fmod(s, 2.0) == 0.0 else refs[1]
                continue
            if kind != TEX_SOLID:
                raise NotImplementedError("NoiseTexture is not restated here")
            return tp[:3]


def _fract(x):                      # f64::fract: self - self.trunc()
    return x - float(math.trunc(x)) if math.isfinite(x) else float("nan")


def _floor(x):
    return float(math.floor(x)) if math.isfinite(x) else x


# --------------------------------------------------------------- integrator
def trace_sample(cam, world, seed, i, j, s):
    """One sample of pixel (i, j): get_ray + ray_colour_tail_call (camera.rs),
    the tail call unrolled into a loop.  Returns ((r, g, b), segments)."""
    W = cam["image_width"]
    g = Rng(seed, j * W + i, s)
    scale = uniform_inclusive_scale(-0.5, 0.5)
    ox = g.uniform(-0.5, scale)
    oy = g.uniform(-0.5, scale)
    ps = add(add(cam["pixel00_loc"], muls(cam["pixel_delta_u"], float(i) + ox)),
             muls(cam["pixel_delta_v"], float(j) + oy))
    if cam["defocus_angle"] <= EPS:
        origin = cam["center"]
    else:
        p = unit_disk(g)
        origin = add(add(cam["center"], muls(cam["defocus_disk_u"], p[0])), muls(cam["defocus_disk_v"], p[2]))
    o, d = origin, sub(ps, origin)
    mult, res = (1.0, 1.0, 1.0), (0.0, 0.0, 0.0)
    bg = cam["background"]
    segments = 0
    for depth in range(cam["max_depth"], -1, -1):
        if depth == 0:
            return add((0.0, 0.0, 0.0), res), segments
        rec = world.hit(o, d)
        segments += 1
        if rec is None:
            return add(mulv(mult, bg), res), segments
        mtype = world.mat_type[rec.mat]
        emitted = world.colour(rec.mat, rec.u, rec.v, rec.p) if mtype == DIFFUSE_LIGHT else (0.0, 0.0, 0.0)
        if mtype == METAL:
            albedo, fuzz = world.mat_params[rec.mat][:3], world.mat_params[rec.mat][3]
            reflected = reflect(normalize(d), rec.normal)
            dirn = add(reflected, muls(unit_sphere(g), fuzz))
            if not dot(dirn, rec.normal) > 0.0:
                return add(mulv(mult, emitted), res), segments
            mult = mulv(mult, albedo)                     # Reflect: mult * attenuation
            o, d = rec.p, dirn
        elif mtype == DIELECTRIC:
            ior = world.mat_params[rec.mat][4]
            ratio = fdiv(1.0, ior) if rec.front else ior
            unit = normalize(d)
            cos_t = fmin(dot(unit, neg(rec.normal)), 1.0)
            sin_t = sqrt(1.0 - cos_t * cos_t)
            if ratio * sin_t > 1.0:
                dirn = reflect(unit, rec.normal)
            else:
                r0 = fdiv(1.0 - ratio, 1.0 + ratio)
                r0 = r0 * r0
                x = 1.0 - cos_t
                refl = r0 + (1.0 - r0) * (x * ((x * x) * (x * x)))   # powi(5)
                dirn = reflect(unit, rec.normal) if refl > g.open01() else refract(unit, rec.normal, ratio)
            mult = mulv(mult, (1.0, 1.0, 1.0))
            o, d = rec.p, dirn
        elif mtype == LAMBERTIAN:
            att = world.colour(rec.mat, rec.u, rec.v, rec.p)
            uvw = Onb(rec.normal)                         # CosinePdf::new(normal)
            if g.standard() < 0.5:                        # MixturePdf::generate
                dirn = world.lights_random(rec.p, g)
            else:
                dirn = uvw.transform(cosine_hemisphere(g))
            cosine_value = fmax(fdiv(dot(normalize(dirn), uvw.w), PI), 0.0)
            pdf = world.lights_pdf(rec.p, dirn) * 0.5 + cosine_value * 0.5
            spdf = fmax(fdiv(dot(rec.normal, normalize(dirn)), PI), 0.0)
            w = divs(muls(att, spdf), pdf)
            res = add(res, mulv(mult, emitted))
            mult = mulv(mult, w)
            o, d = rec.p, dirn
        else:                                             # Invisible / DiffuseLight: scatter None
            return add(mulv(mult, emitted), res), segments
    raise AssertionError("unreachable")
