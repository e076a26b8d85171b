// render_kernel.hpp -- the gfx950 render kernels, templated on precision R
// and on the world query (brute force over an LDS-staged or a global sphere
// list; BVH).
//
// Restates the reference's per-pixel / per-sample loop:
//   render_internal / render_lambda   shared/src/camera.rs:315-388
//   Camera::get_ray                   shared/src/camera.rs:274-293
//   ray_colour_tail_call              shared/src/camera.rs:459-522
// as ONE iterative loop per lane.  Work is cut into ITEMS = (pixel, chunk of
// `chunk` consecutive samples); a wavefront owns a TASK = one 8x8 tile x a
// group of chunks, i.e. a pool of 64 * group items.  Every lane takes an item,
// traces its samples one segment (one world.hit) per loop trip, folds them in
// sample order into the item's partial sum, and when the item is done takes
// the next free item of the pool (ballot + mbcnt: no atomics).  All lanes thus
// share every trip's closest-hit sweep even though the reference's path
// lengths range from 1 to max_depth segments (its t_min = f64::EPSILON makes
// self-intersecting, depth-long paths common).
//
// Chunk sums land in partial[tile][pixel][chunk]; reduce_chunks_kernel folds
// them in chunk order.  Inside a chunk the samples are folded exactly like
// `(0..spp).map(..).fold(Colour::default(), +)` (camera.rs:323-335), so with
// chunk >= spp the f64 result is the reference's fold order bit for bit.
#pragma once

#include <type_traits>

#include "light_grid.hpp"
#include "rtw_device.hpp"
#include "rtw_kernels.h"

namespace rtw {

namespace dev {

// Experiment hooks: every RTW_PROBE_* below expands to nothing in the product
// build; the profiling builds of tools/exp_cost.sh (RTW_EXP) and
// tools/trace_paths.py (RTW_TRACE), tools/lane_profile.py (RTW_PROF) and
// tools/clock_profile.py (RTW_CLOCK) define them in rtw_probes.hpp.
#if defined(RTW_EXP) || defined(RTW_TRACE) || defined(RTW_PROF) || defined(RTW_TIMELINE) || defined(RTW_ABL) || \
    defined(RTW_CLOCK) || defined(RTW_NANORIGIN)
#include "rtw_probes.hpp"
#else
#define RTW_PROBE_NAN_LAMBERT(was, now, obj)
#define RTW_PROBE_HIT_INIT()
#define RTW_PROBE_HIT_RESET()
#define RTW_PROBE_HIT(obj)
#define RTW_PROBE_CLK_INIT()
#define RTW_PROBE_CLK(id)
#define RTW_PROBE_CLK_END()
#define RTW_PROBE_WAVE_BEGIN()
#define RTW_PROBE_WAVE_TASK()
#define RTW_PROBE_WAVE_DRY()
#define RTW_PROBE_WAVE_TRIP()
#define RTW_PROBE_WAVE_END()
#define RTW_PROBE_PLANES()
#define RTW_PROBE_CLOSEST()
#define RTW_PROBE_SEGMENT()
#define RTW_PROBE_LAMBERT_DIR()
#define RTW_PROBE_LIGHT_PDF()
#define RTW_PROBE_SEED()
#define RTW_PROBE_LANES(id)
#define RTW_PROBE_H64()
#define RTW_PROBE_SCATTER64(expr)
#define RTW_PROBE_ABL_DITHER(v)
#define RTW_PROBE_ABL_SELF(hit, ts)
#define RTW_PROBE_ABL_WINNER()
#define RTW_PROBE_ABL_SCATTER(f64)
#endif

template <typename R>
__device__ __forceinline__ V3<R> v3of(const R* a) { return mk(a[0], a[1], a[2]); }

// Plane::get_plane_uv, plane.rs:40-54, on the host-computed per-plane
// constants of the record (rtw_kernels.h kPlaneR): the oracle's plane_uv.
template <typename R>
__device__ __forceinline__ void plane_uv(const R* pl, V3<R> pnt, R& u, R& v) {
    const R mode = pl[12];
    if (mode == (R)0) {
        u = pnt.x;
        v = pnt.z;
        return;
    }
    if (mode == (R)2) {
        u = v = (R)NAN;
        return;
    }
    const V3<R> k = q3(pl, 15);
    const V3<R> vec = pnt - q3(pl, 0);
    const R ct = pl[13], st = pl[14];
    const V3<R> rot = ((vec * ct) + cross(k, vec) * st) + (k * dot(k, vec)) * ((R)1 - ct);
    u = rot.x - trunc_(rot.x);
    v = rot.z - trunc_(rot.z);
}

// One plane, plane.rs:61-76 (one-sided: only rays moving along +n hit it).
// Plane::hit computes the UV before its range test and panics on a
// non-finite one (plane.rs:66-69): counted in *panic (a rare event: one
// atomic at the site, no register kept live).  The UV is not formed
// here: it is NaN for every point of a mode-2 plane, (x, z) for mode 0, and a
// rotation of the finite constants for mode 1 -- non-finite exactly when the
// point is (up to overflow inside the rotation itself, |p| ~ 1e308).
template <typename R, typename PP>
__device__ __forceinline__ bool plane_t(PP pl, V3<R> o, V3<R> d, R tmin, R& t,
                                        unsigned long long* panic) {
    V3<R> n = mk(pl[3], pl[4], pl[5]);
    R denom = dot(d, n);
    if (!(denom > P<R>::kEps)) return false;
    V3<R> op = o - mk(pl[0], pl[1], pl[2]);
    R tt = -P<R>::div_(dot(op, n), denom);
    {
        const V3<R> q = o + d * tt;
        const R mode = pl[12];
        const bool fin = mode == (R)0 ? __builtin_isfinite(q.x) && __builtin_isfinite(q.z)
                                      : mode == (R)1 && __builtin_isfinite(q.x + q.y + q.z);
        if (!fin && panic) atomicAdd(panic, 1ull);
    }
    if (!(tmin <= tt && tt <= (R)INFINITY)) return false;
    t = tt;
    return true;
}

// AABBox::hit, hittable.rs:291-339, over [rs, +inf]: the slab test the
// reference runs before every object's own hit (bounded_hit).  Rust's f64
// max/min ignore a NaN operand like fmax/fmin.
template <typename R, typename PP>
__device__ __forceinline__ bool aabb_hit_ref(PP lo, PP hi, V3<R> o, V3<R> d, R rs) {
    R t0 = P<R>::div_(lo[0] - o.x, d.x), t1 = P<R>::div_(hi[0] - o.x, d.x);
    if (__builtin_signbit(d.x)) { R q = t0; t0 = t1; t1 = q; }
    R tmin = t0, tmax = t1;
    R a0 = P<R>::div_(lo[1] - o.y, d.y), a1 = P<R>::div_(hi[1] - o.y, d.y);
    if (__builtin_signbit(d.y)) { R q = a0; a0 = a1; a1 = q; }
    if (tmax < a0 || tmin > a1) return false;
    tmin = P<R>::max_(tmin, a0);
    tmax = P<R>::min_(tmax, a1);
    a0 = P<R>::div_(lo[2] - o.z, d.z);
    a1 = P<R>::div_(hi[2] - o.z, d.z);
    if (__builtin_signbit(d.z)) { R q = a0; a0 = a1; a1 = q; }
    if (tmax < a0 || tmin > a1) return false;
    tmin = P<R>::max_(tmin, a0);
    tmax = P<R>::min_(tmax, a1);
    return P<R>::max_(rs, tmin) <= P<R>::min_((R)INFINITY, tmax);
}

// aabb_hit_ref on a plane's box (Plane::get_aabbox, plane.rs:218-242: every
// axis pinned at [0, 0] or [-inf, inf]) for a finite ray: an infinite axis
// always yields (-inf, +inf) after the sign swap, which no later max_ / min_
// or comparison changes, so the test reduces to the one pinned axis, q = (0 -
// o_a) / d_a, and hits iff !(q < rs) -- the same quotient and the same
// outcome (NaN included) as the six-division reference sequence (f64: IEEE
// division; f32: a * rcp(b), whose infinities for a zero d_a or an infinite
// a follow the same signs).  Anything else (a non-finite ray, other boxes)
// takes aabb_hit_ref itself.
template <typename R, typename PP>
__device__ __forceinline__ bool aabb_hit_plane(PP lo, PP hi, V3<R> o, V3<R> d, R rs) {
    const bool fin = __builtin_isfinite(o.x) && __builtin_isfinite(o.y) && __builtin_isfinite(o.z) &&
                     __builtin_isfinite(d.x) && __builtin_isfinite(d.y) && __builtin_isfinite(d.z);
    int npin = 0, pin = 0;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        if (lo[a] == (R)0 && hi[a] == (R)0 && !__builtin_signbit(lo[a])) {
            ++npin;
            pin = a;
        } else if (!(lo[a] == (R)-INFINITY && hi[a] == (R)INFINITY)) {
            npin = 4;
        }
    }
    if (!fin || npin > 1) return aabb_hit_ref(lo, hi, o, d, rs);
    if (npin == 0) return true;
    const R oa = pin == 0 ? o.x : (pin == 1 ? o.y : o.z);
    const R da = pin == 0 ? d.x : (pin == 1 ? d.y : d.z);
    const R q = P<R>::div_(lo[pin] - oa, da);
    return !(q < rs);
}

// Transformed<Cuboid>::hit (entities/transformations.rs:14-29, cuboid.rs:50-58)
// on the staged record B (rtw_kernels.h kBoxR), as the oracle's box_hit: the
// ray into object space through the inverse (the direction ALSO gets the
// translation, geometry/src/transformations.rs:112-114 -- the reference's
// behaviour), the closest of the six quads (first minimum wins).
template <typename R>
__device__ __forceinline__ V3<R> mat3_mul(const R* M, V3<R> p) {   // Mul<Vec3> for Matrix3
    return mk(dot(q3(M, 0), p), dot(q3(M, 3), p), dot(q3(M, 6), p));
}
template <typename R>
__device__ __forceinline__ bool box_t_hit(const R* B, V3<R> o, V3<R> d, R tmin, R tmax, R& t, int& quad,
                                          V3<R>& o2, V3<R>& d2) {
    if (B[kBoxOk] == (R)0) return false;
    o2 = mat3_mul(B + kBoxInv, o) + q3(B, kBoxTi);
    d2 = mat3_mul(B + kBoxInv, d) + q3(B, kBoxTi);
    int best = -1;
    R bt = (R)INFINITY;
    for (int k = 0; k < 6; ++k) {
        R tt;
        if (quad_t_hit(B + kQuadR * k, o2, d2, tmin, tmax, tt) && (best < 0 || tt < bt)) {
            bt = tt;
            best = k;
        }
    }
    if (best < 0) return false;
    t = bt;
    quad = best;
    return true;
}

// Closest sphere of a contiguous list [0, n), ids base + k.  Semantics of the
// reference's closest hit: t = near root if it lies in [tmin, inf], else the
// far root (sphere.rs:71-80); the smallest t wins, the lowest id on ties.
//
// f64 (parity mode): the reference's exact arithmetic, divisions included.
template <bool kRobust>
__device__ __forceinline__ void sweep_spheres(const R4<double>* __restrict__ sph, uint32_t n,
                                              int32_t base, V3<double> o, V3<double> d, double tmin,
                                              double& tb, int32_t& best) {
#pragma unroll 2
    for (uint32_t k = 0; k < n; ++k) {
        const R4<double> s = sph[k];
        double t;
        if (sphere_t(mk(s.x, s.y, s.z), s.w, o, d, tmin, t) && (best < 0 || t < tb)) {
            tb = t;
            best = base + (int32_t)k;
        }
    }
}
// f32 (speed mode): the per-sphere test, shared by the brute-force sweep and
// the BVH leaves so both give bit-identical t; every FMA is spelled out so
// that contraction cannot differ between the two call sites.
//
// Closest-approach form (Haines et al., "Precision Improvements for Ray/Sphere
// Intersection", Ray Tracing Gems ch. 7): with f = o - c, the ray's closest
// point to the centre is at tc = -(f.d)/a and l = f + tc d is the offset from
// the centre to it; the discriminant is a (r^2 - l.l).  The reference's
// hb^2 - a c cancels catastrophically in f32 once |f| >> r (C5's 1M-sphere
// field seen from ~700 units: the error exceeds r^2 itself); l.l does not.
// Roots t = tc -/+ sqrt((r^2 - l.l) / a).  Scenes whose extent is small next
// to their radii (C2) keep the cheaper reference form (DevScene::robust = 0,
// chosen per launch by the host).  The range test "t in [tmin, tb)"
// is ONE unsigned compare on u = bits(t) - bits(tmin): for t >= 0 float bits
// are monotonic, while every t < tmin (negative, or in [0, tmin)) and NaN
// maps above bits(+inf) - bits(tmin) >= any live bound.  Since t0 <= t1,
// min_u32(u0, u1) is the near root when it is >= tmin, else the far root
// (sphere.rs:71-80).  A miss gives sqrt(negative) = NaN and so no hit.
template <bool kRobust>
__device__ __forceinline__ uint32_t sphere_u(const R4<float>& s, V3<float> o, V3<float> d, float a,
                                             float ia, uint32_t tminb) {
    const float fx = o.x - s.x, fy = o.y - s.y, fz = o.z - s.z;
    const float hb = __builtin_fmaf(d.z, fz, __builtin_fmaf(d.y, fy, d.x * fx));
    float t0, t1;
    if constexpr (kRobust) {
        const float tc = -hb * ia;
        const float lx = __builtin_fmaf(tc, d.x, fx), ly = __builtin_fmaf(tc, d.y, fy),
                    lz = __builtin_fmaf(tc, d.z, fz);
        const float l2 = __builtin_fmaf(lx, lx, __builtin_fmaf(ly, ly, lz * lz));
        const float h = __builtin_amdgcn_sqrtf((s.w - l2) * ia);   // NaN on a miss
        t0 = tc - h;
        t1 = tc + h;
    } else {
        // the reference's form: c = f.f - r^2, disc = hb^2 - a c
        const float c = __builtin_fmaf(fx, fx, __builtin_fmaf(fy, fy, __builtin_fmaf(fz, fz, -s.w)));
        const float disc = __builtin_fmaf(hb, hb, -(a * c));
        const float sq = __builtin_amdgcn_sqrtf(disc);             // NaN on a miss
        const float nb = -hb * ia;
        t0 = __builtin_fmaf(-sq, ia, nb);
        t1 = __builtin_fmaf(sq, ia, nb);
    }
    return min(__float_as_uint(t0) - tminb, __float_as_uint(t1) - tminb);
}
__device__ __forceinline__ float len2_f32(V3<float> d) {
    return __builtin_fmaf(d.z, d.z, __builtin_fmaf(d.y, d.y, d.x * d.x));
}
// Branch-free body so that the compiler keeps a batch of sphere loads in flight.
template <bool kRobust>
__device__ __forceinline__ void sweep_spheres(const R4<float>* __restrict__ sph, uint32_t n,
                                              int32_t base, V3<float> o, V3<float> d, float tmin,
                                              float& tb, int32_t& best) {
    const float a = len2_f32(d);
    const float ia = __builtin_amdgcn_rcpf(a);
    const uint32_t tminb = __float_as_uint(tmin);
    uint32_t ub = __float_as_uint(tb) - tminb;
#pragma unroll 8
    for (uint32_t k = 0; k < n; ++k) {
        const uint32_t u = sphere_u<kRobust>(sph[k], o, d, a, ia, tminb);
        const bool h = u < ub;
        ub = h ? u : ub;
        best = h ? base + (int32_t)k : best;
    }
    tb = __uint_as_float(ub + tminb);
}

// The same with one sphere id excluded (kOptHit64: the sphere the ray starts on)
template <bool kRobust>
__device__ __forceinline__ void sweep_spheres_excl(const R4<float>* __restrict__ sph, uint32_t n, int32_t base,
                                                   V3<float> o, V3<float> d, float tmin, float& tb, int32_t& best,
                                                   int32_t excl) {
    const float a = len2_f32(d);
    const float ia = __builtin_amdgcn_rcpf(a);
    const uint32_t tminb = __float_as_uint(tmin);
    uint32_t ub = __float_as_uint(tb) - tminb;
#pragma unroll 8
    for (uint32_t k = 0; k < n; ++k) {
        const uint32_t u = sphere_u<kRobust>(sph[k], o, d, a, ia, tminb);
        const bool h = u < ub && base + (int32_t)k != excl;
        ub = h ? u : ub;
        best = h ? base + (int32_t)k : best;
    }
    tb = __uint_as_float(ub + tminb);
}

// Sum of Sphere::pdf_value over the light list in list order
// (HittableList::pdf_value, hittable_list.rs:408-412; sphere.rs:101-111).
// f64: the reference's arithmetic, light by light, for every light an f32
// pre-pass cannot rule out.  A light the ray misses adds exactly +0.0 (the sum
// starts at +0.0), so skipping it changes no bit.  The pre-pass rounds the ray
// and the light to f32 and tests the closest approach l (see light_hit_f32)
// against r + E and the direction (hb <= 0 or the origin inside) with slack,
// E = 2^-18 (|o|_1 + |c|_1 + r): far above the f32 error of l (a few 2^-24
// (|o| + |c|)) and of the f64 decision itself (disc's rounding), so every
// light the f64 test hits stays in.
// li32 (may be null): the same lights rounded to f32 with |radius| (staged in
// LDS by the LDS-world kernels): the pre-pass reads them instead of converting
// the f64 records -- the same f32 values, the same mask
// the pre-pass test of one light {c, |r|} (rounded to f32) against the f32 ray
__device__ __forceinline__ bool light_may_hit(float cx, float cy, float cz, float r, float ox, float oy, float oz,
                                              float dx, float dy, float dz, float ia, float on, float dn) {
    const float fx = ox - cx, fy = oy - cy, fz = oz - cz;
    const float hb = __builtin_fmaf(dz, fz, __builtin_fmaf(dy, fy, dx * fx));
    const float tc = -hb * ia;
    const float lx = __builtin_fmaf(tc, dx, fx), ly = __builtin_fmaf(tc, dy, fy), lz = __builtin_fmaf(tc, dz, fz);
    const float l2 = __builtin_fmaf(lx, lx, __builtin_fmaf(ly, ly, lz * lz));
    const float f2 = __builtin_fmaf(fx, fx, __builtin_fmaf(fy, fy, fz * fz));
    const float e = 0x1p-18f * (on + fabsf(cx) + fabsf(cy) + fabsf(cz) + r);
    const float rr = (r + e) * (r + e);
    // NaN anywhere (a NaN ray): no candidate; the f64 test gives 0 too
    return (l2 <= rr) & ((hb <= 2.0f * e * dn) | (f2 <= rr));
}
// The f32 ray of the pre-pass: o, d rounded, 1 / (d . d), |o|_1, |d|_1
struct LightPre {
    float ox, oy, oz, dx, dy, dz, ia, on, dn;
    __device__ __forceinline__ LightPre(V3<double> o, V3<double> d)
        : ox((float)o.x), oy((float)o.y), oz((float)o.z), dx((float)d.x), dy((float)d.y), dz((float)d.z) {
        ia = __builtin_amdgcn_rcpf(__builtin_fmaf(dx, dx, __builtin_fmaf(dy, dy, dz * dz)));
        on = fabsf(ox) + fabsf(oy) + fabsf(oz);
        dn = fabsf(dx) + fabsf(dy) + fabsf(dz);
    }
    __device__ __forceinline__ bool may_hit(const R4<double>& L) const {
        return light_may_hit((float)L.x, (float)L.y, (float)L.z, fabsf((float)L.w), ox, oy, oz, dx, dy, dz, ia, on, dn);
    }
};

// Inserts x into ids[0..kMax) (ascending; empty entries ~0u) by one
// compare-exchange pass with static indices -- a shifting insertion's dynamic
// register indices compile to 8-way select chains per step -- and returns the
// value that fell off the end (~0u: none did).
template <uint32_t kMax>
__device__ __forceinline__ uint32_t sorted_insert(uint32_t (&ids)[kMax], uint32_t x) {
#pragma unroll
    for (uint32_t q = 0; q < kMax; ++q) {
        const uint32_t a = ids[q];
        ids[q] = min(a, x);
        x = max(a, x);
    }
    return x;
}

// HittableList::pdf_value's sum over the hit lights in LIST order (f64) when
// an acceleration structure finds them in another order: `walk(lo, add)` calls
// add(id) once for every light the ray hits, in any order, and each pass keeps
// the kMax smallest list indices >= lo; their pdfs are added in index order
// and, when the pass had to drop hits, the next pass continues above the last
// index summed.  (A ray skimming C5's flat light layer hits ~10 lights.)
// (R: the sum's type; pdf(id): light id's pdf)
template <typename R, typename Walk, typename Pdf>
__device__ __forceinline__ R lights_sum_ids_in_list_order(Walk&& walk, Pdf&& pdf) {
    constexpr uint32_t kMax = 8;
    R acc = (R)0;
    uint32_t lo = 0;
    for (;;) {
        uint32_t ids[kMax];
#pragma unroll
        for (uint32_t q = 0; q < kMax; ++q) ids[q] = 0xffffffffu;
        bool dropped = false;
        walk([&](uint32_t id) {
            if (id < lo) return;
            // by list index; when full the largest gives way
            if (sorted_insert(ids, id) != 0xffffffffu) dropped = true;
        });
        for (uint32_t q = 0; q < kMax && ids[q] != 0xffffffffu; ++q) acc = acc + pdf(ids[q]);
        if (!dropped) return acc;
        lo = ids[kMax - 1] + 1u;
    }
}
template <typename Walk>
__device__ __forceinline__ double lights_sum_in_list_order(const R4<double>* __restrict__ lights, V3<double> o,
                                                           V3<double> d, Walk&& walk) {
    return lights_sum_ids_in_list_order<double>(walk, [&](uint32_t id) {
        const R4<double> L = lights[id];
        return sphere_pdf_value(mk(L.x, L.y, L.z), L.w, o, d);
    });
}

template <bool kRobust = false>
__device__ __forceinline__ double lights_pdf_sum(const R4<double>* __restrict__ li, uint32_t n,
                                                 V3<double> o, V3<double> d,
                                                 const R4<float>* __restrict__ li32 = nullptr) {
    const float ox = (float)o.x, oy = (float)o.y, oz = (float)o.z;
    const float dx = (float)d.x, dy = (float)d.y, dz = (float)d.z;
    const float a = __builtin_fmaf(dx, dx, __builtin_fmaf(dy, dy, dz * dz));
    const float ia = __builtin_amdgcn_rcpf(a);
    const float on = fabsf(ox) + fabsf(oy) + fabsf(oz);
    const float dn = fabsf(dx) + fabsf(dy) + fabsf(dz);
    double acc = 0.0;
    for (uint32_t base = 0; base < n; base += 32) {
        const uint32_t m = min(32u, n - base);
        uint32_t mask = 0;
        for (uint32_t k = 0; k < m; ++k) {
            float cx, cy, cz, r;
            if (li32) {
                const R4<float> L = li32[base + k];
                cx = L.x;
                cy = L.y;
                cz = L.z;
                r = L.w;
            } else {
                const R4<double> L = li[base + k];
                cx = (float)L.x;
                cy = (float)L.y;
                cz = (float)L.z;
                r = fabsf((float)L.w);
            }
            mask |= (light_may_hit(cx, cy, cz, r, ox, oy, oz, dx, dy, dz, ia, on, dn) ? 1u : 0u) << k;
        }
        while (mask) {
            const uint32_t k = (uint32_t)__builtin_ctz(mask);
            mask &= mask - 1u;
            const R4<double> L = li[base + k];
            acc = acc + sphere_pdf_value(mk(L.x, L.y, L.z), L.w, o, d);
        }
    }
    return acc;
}

// f32 light test: does the ray hit the light sphere with t in [0, inf)?  The
// closest-approach offset l (see sphere_u) gives disc > 0 <=> l.l < r^2
// without cancellation; the far root is >= 0 exactly when tc >= 0 or the
// origin is inside (|f|^2 <= r^2).
template <bool kRobust>
__device__ __forceinline__ bool light_hit_f32(const R4<float>& L, V3<float> o, V3<float> d, float a, float ia) {
    const float fx = o.x - L.x, fy = o.y - L.y, fz = o.z - L.z;
    const float hb = __builtin_fmaf(d.z, fz, __builtin_fmaf(d.y, fy, d.x * fx));
    const float r2 = L.w * L.w;
    if constexpr (kRobust) {
        const float tc = -hb * ia;
        const float lx = __builtin_fmaf(tc, d.x, fx), ly = __builtin_fmaf(tc, d.y, fy),
                    lz = __builtin_fmaf(tc, d.z, fz);
        const float l2 = __builtin_fmaf(lx, lx, __builtin_fmaf(ly, ly, lz * lz));
        const float f2 = __builtin_fmaf(fx, fx, __builtin_fmaf(fy, fy, fz * fz));
        return (l2 < r2) & ((hb <= 0.f) | (f2 <= r2));
    } else {
        // disc = hb^2 - a c > 0 with c = f.f - r^2
        const float c = __builtin_fmaf(fx, fx, __builtin_fmaf(fy, fy, __builtin_fmaf(fz, fz, -r2)));
        const float disc = __builtin_fmaf(hb, hb, -(a * c));
        return (disc > 0.f) & ((hb <= 0.f) | (c <= 0.f));
    }
}
// its solid-angle pdf, 1 / (2 pi (1 - cos_max)) with 1 - cos_max = x / (1 +
// sqrt(1 - x)), x = r^2/d^2 (no cancellation for far lights)
__device__ __forceinline__ float light_pdf_f32(const R4<float>& L, V3<float> o) {
    const float cx = L.x - o.x, cy = L.y - o.y, cz = L.z - o.z;
    const float dist2 = __builtin_fmaf(cx, cx, __builtin_fmaf(cy, cy, cz * cz));
    const float x = L.w * L.w * __builtin_amdgcn_rcpf(dist2);
    const float one_minus_cos = x * __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_sqrtf(1.f - x));
    return __builtin_amdgcn_rcpf(6.283185307179586f * one_minus_cos);
}
// f32: pass 1 finds the lights the ray hits (light_hit_f32, no square root) -- with
// disc > 0 the far root (-hb + sqrt(disc)) / a is >= 0 exactly when hb <= 0
// or c <= 0 -- into a bit mask; pass 2 adds the hit lights' solid-angle pdfs
// in list order.  Most rays hit zero or one light.
template <bool kRobust>
__device__ __forceinline__ float lights_pdf_sum(const R4<float>* __restrict__ li, uint32_t n,
                                                V3<float> o, V3<float> d) {
    const float a = len2_f32(d);
    const float ia = __builtin_amdgcn_rcpf(a);
    float acc = 0.f;
    for (uint32_t base = 0; base < n; base += 32) {
        const uint32_t m = min(32u, n - base);
        uint32_t mask = 0;
#pragma unroll 4
        for (uint32_t k = 0; k < m; ++k) {
            const R4<float> L = li[base + k];
            const bool hit = light_hit_f32<kRobust>(L, o, d, a, ia);
            mask |= (hit ? 1u : 0u) << k;
        }
        while (mask) {
            const uint32_t k = (uint32_t)__builtin_ctz(mask);
            mask &= mask - 1u;
            const R4<float> L = li[base + k];
            acc += light_pdf_f32(L, o);
        }
    }
    return acc;
}

// The same with pass 1 on packed FP32 (v_pk_fma/mul/add_f32: two lights per
// instruction).  lp = the light list as pairs, two R4 per pair {x0, x1, y0,
// y1}, {z0, z1, r0^2, r1^2} (an odd list ends with r^2 = -inf: never hit),
// staged in LDS; each packed lane does exactly light_hit_f32's operations, so
// the mask -- and the sum -- are bit-identical to lights_pdf_sum.
typedef float f2v __attribute__((ext_vector_type(2)));
// `sampled` (>= 0): the light the direction was drawn toward (Sphere::random,
// sphere.rs:113-127) counts whatever the f32 test says: the direction lies in
// its cone, so the reference's f64 test hits it (but at an ulp of the cone's
// edge), while the f32 discriminant can lose the grazing edge directions --
// and a lost light there turns the bounce's pdf to 0 and its weight to 0 / 0
// when the light is below the surface (r04: the f32 mode's surplus NaN
// samples on spheres that overlap no light, tools/nan_origins.py).
template <bool kRobust>
__device__ __forceinline__ float lights_pdf_sum_pk(const R4<float>* __restrict__ li,
                                                   const R4<float>* __restrict__ lp, uint32_t n,
                                                   V3<float> o, V3<float> d, int32_t sampled = -1) {
    const float a = len2_f32(d);
    const float ia = __builtin_amdgcn_rcpf(a);
    const f2v ox = {o.x, o.x}, oy = {o.y, o.y}, oz = {o.z, o.z};
    const f2v dx = {d.x, d.x}, dy = {d.y, d.y}, dz = {d.z, d.z};
    const f2v a2 = {a, a}, ia2 = {ia, ia};
    float acc = 0.f;
    for (uint32_t base = 0; base < n; base += 32) {
        const uint32_t m = min(32u, n - base);
        uint32_t mask = 0;
#pragma unroll 2
        for (uint32_t k = 0; k < m; k += 2) {
            const R4<float> A = lp[base + k], B = lp[base + k + 1];
            const f2v fx = ox - f2v{A.x, A.y}, fy = oy - f2v{A.z, A.w}, fz = oz - f2v{B.x, B.y};
            const f2v r2 = {B.z, B.w};
            const f2v hb = __builtin_elementwise_fma(dz, fz, __builtin_elementwise_fma(dy, fy, dx * fx));
            bool h0, h1;
            if constexpr (kRobust) {
                const f2v tc = -hb * ia2;
                const f2v lx = __builtin_elementwise_fma(tc, dx, fx), ly = __builtin_elementwise_fma(tc, dy, fy),
                          lz = __builtin_elementwise_fma(tc, dz, fz);
                const f2v l2 = __builtin_elementwise_fma(lx, lx, __builtin_elementwise_fma(ly, ly, lz * lz));
                const f2v f2 = __builtin_elementwise_fma(fx, fx, __builtin_elementwise_fma(fy, fy, fz * fz));
                h0 = (l2.x < r2.x) & ((hb.x <= 0.f) | (f2.x <= r2.x));
                h1 = (l2.y < r2.y) & ((hb.y <= 0.f) | (f2.y <= r2.y));
            } else {
                const f2v c = __builtin_elementwise_fma(fx, fx, __builtin_elementwise_fma(fy, fy,
                                                                __builtin_elementwise_fma(fz, fz, -r2)));
                const f2v disc = __builtin_elementwise_fma(hb, hb, -(a2 * c));
                h0 = (disc.x > 0.f) & ((hb.x <= 0.f) | (c.x <= 0.f));
                h1 = (disc.y > 0.f) & ((hb.y <= 0.f) | (c.y <= 0.f));
            }
            mask |= ((h0 ? 1u : 0u) | (h1 ? 2u : 0u)) << k;
        }
        if ((uint32_t)(sampled - (int32_t)base) < 32u) mask |= 1u << (sampled - (int32_t)base);
        while (mask) {
            const uint32_t k = (uint32_t)__builtin_ctz(mask);
            mask &= mask - 1u;
            const R4<float> L = li[base + k];
            acc += light_pdf_f32(L, o);
        }
    }
    return acc;
}

// ---------------------------------------------------------------------------
// BVH closest hit (RTW_ACCEL_BVH).  Box tests only cull; every surviving
// sphere goes through the same per-sphere arithmetic as the brute-force
// sweep, and the lowest id wins ties, so the result is the brute-force result.
// ---------------------------------------------------------------------------
template <typename R, bool kRobust>
struct SphereTester;

__device__ __forceinline__ float bperm_f(float x, int32_t src) {
    return __int_as_float(__builtin_amdgcn_ds_bpermute(src << 2, __float_as_int(x)));
}
__device__ __forceinline__ int32_t bperm_i(int32_t x, int32_t src) { return __builtin_amdgcn_ds_bpermute(src << 2, x); }
__device__ __forceinline__ float bperm_any(float x, int32_t src) { return bperm_f(x, src); }
__device__ __forceinline__ double bperm_any(double x, int32_t src);
__device__ __forceinline__ double bperm_d(double x, int32_t src) {
    const uint64_t b = (uint64_t)__double_as_longlong(x);
    const uint32_t lo = (uint32_t)bperm_i((int32_t)(uint32_t)b, src), hi = (uint32_t)bperm_i((int32_t)(b >> 32), src);
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}
__device__ __forceinline__ double bperm_any(double x, int32_t src) { return bperm_d(x, src); }

template <bool kRobust>
struct SphereTester<double, kRobust> {   // exact reference arithmetic (sphere.rs:61-80)
    V3<double> o, d;
    double tmin, tb;
    int32_t best;
    __device__ __forceinline__ double bound() const { return tb; }
    // the ray and running result of lane `src` (subtree stealing)
    __device__ __forceinline__ void take(int32_t src) {
        o = mk(bperm_d(o.x, src), bperm_d(o.y, src), bperm_d(o.z, src));
        d = mk(bperm_d(d.x, src), bperm_d(d.y, src), bperm_d(d.z, src));
        tb = bperm_d(tb, src);
        best = bperm_i(best, src);
    }
    // returns whether the sphere is hit at all (t in [tmin, inf])
    __device__ __forceinline__ bool test_hit(const R4<double>& s, int32_t id) {
        double t;
        const bool hit = sphere_t(mk(s.x, s.y, s.z), s.w, o, d, tmin, t);
        if (hit && (best < 0 || t < tb || (t == tb && id < best))) {
            tb = t;
            best = id;
        }
        return hit;
    }
    __device__ __forceinline__ void test(const R4<double>& s, int32_t id) { (void)test_hit(s, id); }
};

template <bool kRobust>
struct SphereTester<float, kRobust> {    // the f32 sweep's arithmetic (see sphere_u)
    V3<float> o, d;
    float a, ia;
    uint32_t tminb, ub;
    int32_t best;
    __device__ __forceinline__ float bound() const { return __uint_as_float(ub + tminb); }
    // (ub, best) as one unsigned key whose order is test()'s: ub first, then the
    // id in signed order (best = -1 below every id); the minimum over partial
    // traversals of one ray is the single traversal's result (subtree stealing)
    __device__ __forceinline__ uint64_t key() const {
        return ((uint64_t)ub << 32) | ((uint32_t)best ^ 0x80000000u);
    }
    __device__ __forceinline__ void from_key(uint64_t k) {
        ub = (uint32_t)(k >> 32);
        best = (int32_t)((uint32_t)k ^ 0x80000000u);
    }
    // the ray and running result of lane `src` (every lane of the wave takes
    // part: ds_bpermute reads the source lane's registers)
    __device__ __forceinline__ void take(int32_t src) {
        o = mk(bperm_f(o.x, src), bperm_f(o.y, src), bperm_f(o.z, src));
        d = mk(bperm_f(d.x, src), bperm_f(d.y, src), bperm_f(d.z, src));
        ub = (uint32_t)bperm_i((int32_t)ub, src);
        best = bperm_i(best, src);
        a = len2_f32(d);
        ia = __builtin_amdgcn_rcpf(a);
    }
    __device__ __forceinline__ void test(const R4<float>& s, int32_t id) {
        const uint32_t u = sphere_u<kRobust>(s, o, d, a, ia, tminb);
        const bool upd = u < ub || (u == ub && id < best);
        ub = upd ? u : ub;
        best = upd ? id : best;
    }
    // returns whether the sphere is hit at all (t in [tmin, inf])
    __device__ __forceinline__ bool test_hit(const R4<float>& s, int32_t id) {
        const uint32_t u = sphere_u<kRobust>(s, o, d, a, ia, tminb);
        const bool upd = u < ub || (u == ub && id < best);
        ub = upd ? u : ub;
        best = upd ? id : best;
        return u <= 0x7f800000u - tminb;
    }
};

__device__ __forceinline__ double inv_(double x) { return 1.0 / x; }
__device__ __forceinline__ float inv_(float x) { return __builtin_amdgcn_rcpf(x); }

// Near-child-first traversal with a per-lane stack in LDS (stk[entry * 64]).
// Slab test on padded child boxes against [0, tb].
template <typename R, typename TT>
__device__ __forceinline__ void bvh_traverse(const DevScene<R>& sc, int32_t base, V3<R> o, V3<R> d,
                                             TT& T, int32_t* __restrict__ stk,
                                             uint32_t& nvis, uint32_t& ntest, bool skip) {
    if (skip) return;
    const R ix = inv_(d.x), iy = inv_(d.y), iz = inv_(d.z);
    const R oix = o.x * ix, oiy = o.y * iy, oiz = o.z * iz;
    const BvhNode<R>* __restrict__ nodes = sc.bvh;
    int32_t sp = 0;
    int32_t node = 0;
    for (;;) {
        if (node >= 0) {
            ++nvis;
            const BvhNode<R>& nd = nodes[node];
            const R tb = T.bound();
            R tn[2], tf[2];
#pragma unroll
            for (int c = 0; c < 2; ++c) {
                const R x0 = nd.lo_x[c] * ix - oix, x1 = nd.hi_x[c] * ix - oix;
                const R y0 = nd.lo_y[c] * iy - oiy, y1 = nd.hi_y[c] * iy - oiy;
                const R z0 = nd.lo_z[c] * iz - oiz, z1 = nd.hi_z[c] * iz - oiz;
                tn[c] = fmax(fmax(fmin(x0, x1), fmin(y0, y1)), fmax(fmin(z0, z1), (R)0));
                tf[c] = fmin(fmin(fmax(x0, x1), fmax(y0, y1)), fmin(fmax(z0, z1), tb));
            }
            const bool h0 = tn[0] <= tf[0], h1 = tn[1] <= tf[1];
            const int32_t c0 = nd.child[0], c1 = nd.child[1];
            if (h0 && h1) {
                const bool first0 = tn[0] <= tn[1];
                stk[sp * 64] = first0 ? c1 : c0;
                ++sp;
                node = first0 ? c0 : c1;
            } else if (h0) {
                node = c0;
            } else if (h1) {
                node = c1;
            } else {
                if (sp == 0) break;
                --sp;
                node = stk[sp * 64];
            }
        } else {
            const uint32_t code = (uint32_t)~node;
            const uint32_t first = code >> 4, cnt = code & 15u;
            for (uint32_t k = 0; k < cnt; ++k)
                T.test(sc.bsph[first + k], base + (int32_t)sc.bid[first + k]);
            ntest += cnt;
            if (sp == 0) break;
            --sp;
            node = stk[sp * 64];
        }
    }
}

// Test a parked leaf (<= 15 spheres, contiguous in bsph/bid) in groups of
// four: each group's slots are fetched at once (indices clamped to the leaf,
// so a short group re-tests its last sphere -- a no-op: same t, same id, and
// ties only move to a LOWER id) and tested without a data-dependent trip
// count.  With the default 4-sphere leaves there is exactly one group.
// f64 leaves: an f32 pre-pass (sphere_may_hit: the light pre-pass of
// lights_pdf_sum on {c, r^2}, with (r + e)^2 <= r^2 + e (r^2 + 1) + e^2) masks
// the spheres the ray may hit; only those get the f64 test, each read from
// the f64 leaf array -- the closest (t, id) does not depend on the order or on
// spheres the ray misses.  The pre-pass reads the leaf spheres rounded to f32
// (DevScene::bsph32, staged in LDS by the LDS-world kernel: half the bytes of
// the f64 array, which stays in HBM / L1 for the few candidates).  Holding the
// four f64 spheres across the mask loop instead spilled 78 VGPRs and ran
// slower.
__device__ __forceinline__ bool sphere_may_hit(const R4<float>& S, float ox, float oy, float oz, float dx,
                                               float dy, float dz, float ia, float on, float dn) {
    const float cx = S.x, cy = S.y, cz = S.z, r2 = S.w;   // the f64 sphere rounded to f32 (bsph32)
    const float fx = ox - cx, fy = oy - cy, fz = oz - cz;
    const float hb = __builtin_fmaf(dz, fz, __builtin_fmaf(dy, fy, dx * fx));
    const float tc = -hb * ia;
    const float lx = __builtin_fmaf(tc, dx, fx), ly = __builtin_fmaf(tc, dy, fy), lz = __builtin_fmaf(tc, dz, fz);
    const float l2 = __builtin_fmaf(lx, lx, __builtin_fmaf(ly, ly, lz * lz));
    const float f2 = __builtin_fmaf(fx, fx, __builtin_fmaf(fy, fy, fz * fz));
    const float e = 0x1p-18f * (on + fabsf(cx) + fabsf(cy) + fabsf(cz) + 0.5f * (r2 + 1.0f));
    const float rr = __builtin_fmaf(e, r2 + 1.0f + e, r2);
    return (l2 <= rr) & ((hb <= 2.0f * e * dn) | (f2 <= rr));
}
template <typename R, typename TT>
__device__ __forceinline__ void test_leaf(const DevScene<R>& sc, int32_t base, int32_t leaf,
                                          TT& T, uint32_t& ntest) {
    const uint32_t code = (uint32_t)~leaf;
    const uint32_t first = code >> 4, cnt = code & 15u;
    if constexpr (sizeof(R) == 8) {
        const float ox = (float)T.o.x, oy = (float)T.o.y, oz = (float)T.o.z;
        const float dx = (float)T.d.x, dy = (float)T.d.y, dz = (float)T.d.z;
        const float ia = __builtin_amdgcn_rcpf(__builtin_fmaf(dx, dx, __builtin_fmaf(dy, dy, dz * dz)));
        const float on = fabsf(ox) + fabsf(oy) + fabsf(oz), dn = fabsf(dx) + fabsf(dy) + fabsf(dz);
        uint32_t mask = 0;
        for (uint32_t k = 0; k < cnt; ++k)
            mask |= (sphere_may_hit(sc.bsph32[first + k], ox, oy, oz, dx, dy, dz, ia, on, dn) ? 1u : 0u) << k;
        while (mask) {
            const uint32_t k = (uint32_t)__builtin_ctz(mask);
            mask &= mask - 1u;
#if RTW_EXP_LEAF64_LOAD2
            // (timing experiment) the candidate loaded twice, the second load's
            // address depending on the first's value: the price of one dependent
            // global load in the leaf loop (same values, same image)
            {
                const R4<double> s1 = sc.bsph[first + k];
                uint32_t z;
                asm volatile("v_and_b32 %0, 0, %1" : "=v"(z) : "v"((uint32_t)__double_as_longlong(s1.x)));
                T.test(sc.bsph[first + k + z], base + (int32_t)sc.bid[first + k]);
            }
#else
            T.test(sc.bsph[first + k], base + (int32_t)sc.bid[first + k]);
#endif
        }
        ntest += cnt;
        return;
    }
    for (uint32_t g0 = 0; g0 < cnt; g0 += 4) {
        R4<R> s[4];
        int32_t id[4];
#pragma unroll
        for (uint32_t k = 0; k < 4; ++k) {
            const uint32_t i = first + min(g0 + k, cnt - 1);
            s[k] = sc.bsph[i];
            id[k] = (int32_t)sc.bid[i];
        }
        if constexpr (sizeof(R) == 4) {
            asm volatile("" : "+v"(s[0].x), "+v"(s[1].x), "+v"(s[2].x), "+v"(s[3].x), "+v"(id[0]), "+v"(id[1]),
                         "+v"(id[2]), "+v"(id[3]));
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) T.test(s[k], base + id[k]);
    }
    ntest += cnt;
}

// "While-while" traversal with leaf postponing (Aila & Laine 2009): inner
// nodes and leaves are processed in separate wave-uniform phases, so the
// SIMD never runs the box-test and the sphere-test code under one divergent
// branch.  A lane that reaches a leaf parks it and keeps descending until it
// holds a second leaf; the inner phase ends when every lane holds a leaf (or
// is done), then all parked leaves are tested together.
//
// Both precisions cull on the f32 tree (sc.bvh32).  An f64 ray (the parity
// mode) is rounded to f32 and every slab interval is widened by a bound on
// the error of that f32 arithmetic, so a box the exact f64 ray meets within
// [0, tb] is never culled; the spheres that survive are tested in f64 as
// before (the result is the brute-force result, bit for bit).  With ix the
// f32 reciprocal (1 ulp) of the rounded direction, o and d rounded (2^-24),
// each slab parameter t = (b - o) / d comes out within
// |t| 2^-22 + |o ix| 2^-22.9 of its exact value; the interval [tn, tf] is
// widened to [tn (1 - 2^-20) - s, tf (1 + 2^-20) + s], s = 2^-20 max |o ix|,
// and the bound tb is rounded up to f32.
__device__ __forceinline__ const BvhNode<float>* cull_nodes(const DevScene<float>& sc) { return sc.bvh; }
__device__ __forceinline__ const BvhNode<float>* cull_nodes(const DevScene<double>& sc) { return sc.bvh32; }
__device__ __forceinline__ float cull_bound(float t) { return t; }
__device__ __forceinline__ float cull_bound(double t) {   // t rounded up to f32
    const float f = (float)t;
    return (double)f < t ? __uint_as_float(__float_as_uint(f) + 1u) : f;   // t > 0
}
// RTW_NT_NODES (experiment): the while-while traversal's node loads non-temporal
// (trees outside LDS: C3 / C5), so that streaming a large tree through L2 does
// not evict the light grid the walk reads
// RTW_COOP_ADAPT: the f64 cooperative walk sizes its pieces per trip (below
// the tuned grid_piece) so the wave's pending cells fill its lanes
#ifndef RTW_COOP_ADAPT
#define RTW_COOP_ADAPT 1
#endif
constexpr uint32_t kCoopAdaptMin = 4;   // the shortest adaptive piece (cells)
// RTW_COOP_DEAL: the f64 cooperative walk deals its owners' candidate pdfs to
// the whole wave (lights_pdf_grid_coop_list)
#ifndef RTW_COOP_DEAL
#define RTW_COOP_DEAL 1
#endif
// RTW_GRID_REC: the cooperative light-grid walks read the cell records
// (DevScene::lg_rec: one 64-byte load per cell) instead of the cell's range
// and then each light (0: the range walk, for A/B)
#ifndef RTW_GRID_REC
#define RTW_GRID_REC 1
#endif
#ifndef RTW_NT_NODES
#define RTW_NT_NODES 0
#endif
__device__ __forceinline__ BvhNode<float> load_node(const BvhNode<float>* __restrict__ nodes, int32_t i) {
    if constexpr (RTW_NT_NODES != 0) {
        static_assert(sizeof(BvhNode<float>) == 64, "node = 4 x 16 B");
        typedef float f4v __attribute__((ext_vector_type(4)));
        const f4v* q = reinterpret_cast<const f4v*>(nodes + i);
        const f4v a = __builtin_nontemporal_load(q), b = __builtin_nontemporal_load(q + 1),
                  c = __builtin_nontemporal_load(q + 2), e = __builtin_nontemporal_load(q + 3);
        BvhNode<float> n;
        n.lo_x[0] = a.x; n.lo_x[1] = a.y; n.lo_y[0] = a.z; n.lo_y[1] = a.w;
        n.lo_z[0] = b.x; n.lo_z[1] = b.y; n.hi_x[0] = b.z; n.hi_x[1] = b.w;
        n.hi_y[0] = c.x; n.hi_y[1] = c.y; n.hi_z[0] = c.z; n.hi_z[1] = c.w;
        n.child[0] = __float_as_int(e.x); n.child[1] = __float_as_int(e.y);
        return n;
    } else {
        return nodes[i];
    }
}
template <typename R, typename TT>
__device__ __forceinline__ void bvh_traverse_ww(const DevScene<R>& sc, int32_t base, V3<R> o, V3<R> d,
                                                TT& T, int32_t* __restrict__ stk,
                                                uint32_t& nvis, uint32_t& ntest, bool skip) {
    constexpr int32_t kDone = 0x7fffffff;
    constexpr bool kWide = sizeof(R) == 8;   // f64 ray on the f32 tree: widened intervals
    const float ix = inv_((float)d.x), iy = inv_((float)d.y), iz = inv_((float)d.z);
    const float oix = (float)o.x * ix, oiy = (float)o.y * iy, oiz = (float)o.z * iz;
    // fmaxf drops a NaN (0 x inf: that slab is unbounded anyway); an infinite
    // o ix (a zero direction component) keeps every box: correct, only slow
    const float slack = kWide ? 0x1p-20f * fmaxf(fmaxf(fabsf(oix), fabsf(oiy)), fmaxf(fabsf(oiz), 0.0f)) : 0.0f;
    float tbw = kWide ? cull_bound(T.bound()) : 0.0f;   // kWide: tb as the culling bound, per leaf phase
    const BvhNode<float>* __restrict__ nodes = cull_nodes(sc);
    // b ix - o ix: fused in the f64 build too (built without contraction)
    auto slab = [](float b, float i, float oi) {
        if constexpr (kWide) return __builtin_fmaf(b, i, -oi);
        else return b * i - oi;
    };
    int32_t sp = 0;
    int32_t node = skip ? kDone : 0;   // inner node index, leaf code (< 0) or kDone
    int32_t leaf = 0;   // parked leaf code, 0 = none
    for (;;) {
        for (;;) {
            if (node < 0 && leaf == 0) {   // park the leaf, continue with the stack
                leaf = node;
                node = sp ? stk[--sp * 64] : kDone;
            }
            const bool inner = node >= 0 && node != kDone;
            if (!__any(inner) || __all(leaf != 0 || node == kDone)) break;
            if (inner) {
                RTW_PROBE_LANES(1);
                ++nvis;
                const BvhNode<float> nd = load_node(nodes, node);
                const float tb = kWide ? tbw : (float)T.bound();
                float tn[2], tf[2];
#pragma unroll
                for (int c = 0; c < 2; ++c) {
                    const float x0 = slab(nd.lo_x[c], ix, oix), x1 = slab(nd.hi_x[c], ix, oix);
                    const float y0 = slab(nd.lo_y[c], iy, oiy), y1 = slab(nd.hi_y[c], iy, oiy);
                    const float z0 = slab(nd.lo_z[c], iz, oiz), z1 = slab(nd.hi_z[c], iz, oiz);
                    tn[c] = fmaxf(fmaxf(fminf(x0, x1), fminf(y0, y1)), fmaxf(fminf(z0, z1), 0.0f));
                    tf[c] = fminf(fminf(fmaxf(x0, x1), fmaxf(y0, y1)), fminf(fmaxf(z0, z1), tb));
                    if constexpr (kWide) {
                        tn[c] = __builtin_fmaf(tn[c], 1.0f - 0x1p-20f, -slack);
                        tf[c] = __builtin_fmaf(tf[c], 1.0f + 0x1p-20f, slack);
                    }
                }
                const bool h0 = tn[0] <= tf[0], h1 = tn[1] <= tf[1];
                const int32_t c0 = nd.child[0], c1 = nd.child[1];
                if (h0 && h1) {
                    const bool first0 = tn[0] <= tn[1];
                    stk[sp * 64] = first0 ? c1 : c0;
                    ++sp;
                    node = first0 ? c0 : c1;
                } else if (h0 | h1) {
                    node = h0 ? c0 : c1;
                } else {
                    node = sp ? stk[--sp * 64] : kDone;
                }
            }
        }
        if (!__any(leaf != 0)) break;   // no parked leaves: every lane is done
        if (leaf != 0) {
            RTW_PROBE_LANES(2);
            test_leaf(sc, base, leaf, T, ntest);
            leaf = 0;
            if constexpr (kWide) tbw = cull_bound(T.bound());
        }
    }
}

__device__ __forceinline__ uint32_t sign_bit(float x) { return __float_as_uint(x) >> 31; }
__device__ __forceinline__ int32_t link_of(float x) { return (int32_t)__float_as_uint(x); }
__device__ __forceinline__ int32_t link_of(double x) { return (int32_t)__double_as_longlong(x); }
__device__ __forceinline__ uint32_t sign_bit(double x) {
    return (uint32_t)(__double_as_longlong(x) >> 63) & 1u;
}

// Fetch a whole 4-wide node.  For f32 the eight 16-B loads are issued back
// to back and completed together (the empty asm takes every word as an
// operand); left alone, the scheduler interleaves them with the slab tests
// and waits for each child's second half separately -- four dependent memory
// round trips per visit instead of one.
__device__ __forceinline__ void load_node4(const Bvh4Node<float>& nd, R4<float> (&A)[4], R4<float> (&B)[4]) {
    typedef float f4 __attribute__((ext_vector_type(4)));
    const f4* p = reinterpret_cast<const f4*>(&nd);
    f4 v0 = p[0], v1 = p[1], v2 = p[2], v3 = p[3], v4 = p[4], v5 = p[5], v6 = p[6], v7 = p[7];
    asm volatile("" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7));
    const f4 v[8] = {v0, v1, v2, v3, v4, v5, v6, v7};
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        A[c] = R4<float>{v[c].x, v[c].y, v[c].z, v[c].w};
        B[c] = R4<float>{v[4 + c].x, v[4 + c].y, v[4 + c].z, v[4 + c].w};
    }
}
__device__ __forceinline__ void load_node4(const Bvh4Node<double>& nd, R4<double> (&A)[4], R4<double> (&B)[4]) {
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        A[c] = nd.a[c];
        B[c] = nd.b[c];
    }
}

// 4-wide version of bvh_traverse_ww on the octant copies of the tree
// (Bvh4Node): the ray's octant picks the copy, whose children are already in
// front-to-back order and whose slab planes are already near/far for this
// octant.  The first hit child is visited next; the other hit children are
// pushed far-to-near (each store is unconditional, only the stack pointer
// advance is predicated, so a visit has no divergent branch).  The stack
// holds at most sc.bvh4_stack entries (host-computed bound) and is written
// one past its top.
template <typename R, typename TT>
__device__ __forceinline__ void bvh4_traverse(const DevScene<R>& sc, int32_t base, V3<R> o, V3<R> d,
                                              TT& T, int32_t* __restrict__ stk,
                                              uint32_t& nvis, uint32_t& ntest, bool skip) {
    constexpr int32_t kDone = 0x7fffffff;
    const R ix = inv_(d.x), iy = inv_(d.y), iz = inv_(d.z);
    const R oix = o.x * ix, oiy = o.y * iy, oiz = o.z * iz;
    const uint32_t oct = sign_bit(ix) | (sign_bit(iy) << 1) | (sign_bit(iz) << 2);
    const Bvh4Node<R>* __restrict__ nodes = sc.bvh4 + oct * sc.n_nodes4;
    int32_t sp = 0;
    int32_t node = skip ? kDone : 0;   // inner node index, leaf code (< 0) or kDone
    int32_t leaf = 0;   // parked leaf code, 0 = none
    for (;;) {
        for (;;) {
            if (node < 0 && leaf == 0) {   // park the leaf, continue with the stack
                leaf = node;
                node = sp ? stk[--sp * 64] : kDone;
            }
            const bool inner = node >= 0 && node != kDone;
            if (!__any(inner) || __all(leaf != 0 || node == kDone)) break;
            if (inner) {
                ++nvis;
                R4<R> NA[4], NB[4];
                load_node4(nodes[node], NA, NB);
                const R tb = T.bound();
                bool h[4];
                int32_t ch[4];
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    const R4<R> A = NA[c], B = NB[c];
                    const R xn = A.x * ix - oix, yn = A.y * iy - oiy, zn = A.z * iz - oiz;
                    const R xf = A.w * ix - oix, yf = B.x * iy - oiy, zf = B.y * iz - oiz;
                    const R tn = fmax(fmax(xn, yn), fmax(zn, (R)0));
                    const R tf = fmin(fmin(xf, yf), fmin(zf, tb));
                    h[c] = tn <= tf;
                    ch[c] = link_of(B.z);
                }
                const int32_t c0 = ch[0], c1 = ch[1], c2 = ch[2], c3 = ch[3];
                stk[sp * 64] = c3;
                sp += (h[3] && (h[0] || h[1] || h[2])) ? 1 : 0;
                stk[sp * 64] = c2;
                sp += (h[2] && (h[0] || h[1])) ? 1 : 0;
                stk[sp * 64] = c1;
                sp += (h[1] && h[0]) ? 1 : 0;
                if (h[0] | h[1] | h[2] | h[3])
                    node = h[0] ? c0 : (h[1] ? c1 : (h[2] ? c2 : c3));
                else
                    node = sp ? stk[--sp * 64] : kDone;
            }
        }
        if (!__any(leaf != 0)) break;   // no parked leaves: every lane is done
        if (leaf != 0) {
            test_leaf(sc, base, leaf, T, ntest);
            leaf = 0;
        }
    }
}

// Subtree stealing: the result slots of one wave's rays in LDS.  f32: one
// u64 key per ray (SphereTester<float>::key, folded with an atomic min).  f64:
// the t bits (t >= t_min > 0: their unsigned order is t's) and the id, folded
// in two wave-synchronous steps -- an atomic min of t, then the id of a lane
// whose t is the new minimum (stored by the lane that lowered it, atomic min
// among equal t) -- the tester's order (smallest t, then lowest id, best = -1
// above every id).  fold() must be called by every lane of the wave
// (`on` selects the folding lanes).
template <typename R>
struct StealSlots;
template <>
struct StealSlots<float> {
    unsigned long long* key;
    __device__ __forceinline__ explicit StealSlots(unsigned char* area)
        : key(reinterpret_cast<unsigned long long*>(area)) {}
    template <typename TT>
    __device__ __forceinline__ void init(uint32_t lane, const TT& T) { key[lane] = T.key(); }
    template <typename TT>
    __device__ __forceinline__ void fold(bool on, int32_t owner, TT& T, bool share) {
        if (on) {
            const uint64_t k = T.key();
            const uint64_t prev = atomicMin(key + owner, (unsigned long long)k);
            if (share) T.from_key(prev < k ? prev : k);
        }
    }
    template <typename TT>
    __device__ __forceinline__ void refresh(bool on, int32_t owner, TT& T) {
        if (on) {
            const uint64_t ko = key[owner];
            if (ko < T.key()) T.from_key(ko);
        }
    }
    template <typename TT>
    __device__ __forceinline__ void result(uint32_t lane, TT& T) { T.from_key(key[lane]); }
};
template <>
struct StealSlots<double> {
    // per ray: the exact result (t bits, id) -- lowered only by full folds, so
    // its id always belongs to its t -- and a culling bound (t bits) that the
    // lanes on the ray lower after every leaf phase with one atomic
    unsigned long long* tb;
    uint32_t* id;
    unsigned long long* cull;
    // a lane whose bound came from another lane's hit holds no hit at that t:
    // its id is above every real id (ties at that t go to the real hit; the
    // full fold's id step never picks it)
    static constexpr int32_t kForeign = 0x7fffffff;
    __device__ __forceinline__ explicit StealSlots(unsigned char* area)
        : tb(reinterpret_cast<unsigned long long*>(area)), id(reinterpret_cast<uint32_t*>(area + 64 * 8)),
          cull(reinterpret_cast<unsigned long long*>(area + 64 * 12)) {}
    static __device__ __forceinline__ uint64_t bits(double t) { return (uint64_t)__double_as_longlong(t); }
    template <typename TT>
    __device__ __forceinline__ void init(uint32_t lane, const TT& T) {
        tb[lane] = bits(T.tb);
        id[lane] = (uint32_t)T.best;
        cull[lane] = bits(T.tb);
    }
    // the exact (t, id) into the owner's result, in the tester's order
    // (smallest t, then lowest id; best = -1 above every id): an atomic min of
    // t, then the id of a lane whose t is the new minimum (stored by the lane
    // that lowered it, atomic min among equal t).  Every lane of the wave calls
    // it (`on` selects the folding lanes).
    template <typename TT>
    __device__ __forceinline__ void fold(bool on, int32_t owner, TT& T, bool) {
        const uint64_t t = bits(T.tb);
        bool lowered = false;
        if (on) {
            lowered = t < atomicMin(tb + owner, (unsigned long long)t);
            atomicMin(cull + owner, (unsigned long long)t);
        }
        __builtin_amdgcn_wave_barrier();
        const uint64_t cur = on ? tb[owner] : 0;
        if (on && t == cur && lowered) id[owner] = (uint32_t)T.best;
        __builtin_amdgcn_wave_barrier();
        if (on && t == cur) atomicMin(id + owner, (uint32_t)T.best);
    }
    // after a leaf phase: share the bound only (one returning atomic); a lane
    // whose t is above the ray's bound takes it with the foreign id
    template <typename TT>
    __device__ __forceinline__ void share(bool on, int32_t owner, TT& T) {
        if (on) {
            const uint64_t t = bits(T.tb);
            const uint64_t prev = atomicMin(cull + owner, (unsigned long long)t);
            if (prev < t) {
                T.tb = __longlong_as_double((long long)prev);
                T.best = kForeign;
            }
        }
    }
    template <typename TT>
    __device__ __forceinline__ void refresh(bool on, int32_t owner, TT& T) {
        if (on) {
            const uint64_t t = cull[owner];
            if (t < bits(T.tb)) {
                T.tb = __longlong_as_double((long long)t);
                T.best = kForeign;
            }
        }
    }
    template <typename TT>
    __device__ __forceinline__ void result(uint32_t lane, TT& T) {
        T.tb = __longlong_as_double((long long)tb[lane]);
        T.best = (int32_t)id[lane];
    }
};
template <typename TT>
__device__ __forceinline__ void steal_share(StealSlots<float>& S, bool on, int32_t owner, TT& T) {
    S.fold(on, owner, T, true);
}
template <typename TT>
__device__ __forceinline__ void steal_share(StealSlots<double>& S, bool on, int32_t owner, TT& T) {
    S.share(on, owner, T);
}

// bvh_traverse_ww with intra-wave subtree stealing.  A lane with nothing left
// to traverse -- its ray done, or never started (the own-sphere shortcut) --
// takes the bottom entry of another lane's stack (the largest subtree that
// lane has postponed) together with that lane's ray and running result, and
// traverses it as its own; lanes pair up by rank (the k-th idle lane with the
// k-th lane holding stack entries) through 64 rendezvous bytes in LDS, the ray
// moves with ds_bpermute.  Every lane on a ray folds its result into the ray
// owner's slot after each leaf phase and culls with the minimum so far (the
// bound is shared), and a finished partial traversal is folded before the
// lane steals again; the owner reads the minimum at the end.  Box tests only
// cull and the slot order is the tester's (smallest t, then lowest id), so
// the result is the single traversal's bit for bit (tests: BVH == brute
// force, f64 == oracle).  f64 rays cull on the f32 tree with widened slab
// intervals exactly as bvh_traverse_ww.  tools/steal_sim.cpp (lockstep
// simulation on C2 ray batches): 17.0 -> 8.4 inner passes and 3.9 -> 1.9
// leaf passes per 64 segments.
template <typename R, typename TT>
__device__ __forceinline__ void bvh_traverse_steal(const DevScene<R>& sc, int32_t base, TT& T,
                                                   int32_t* __restrict__ stk_wave, uint32_t lane,
                                                   unsigned char* __restrict__ steal_area, uint32_t& nvis,
                                                   uint32_t& ntest, bool skip) {
    constexpr int32_t kDone = 0x7fffffff;
    constexpr bool kWide = sizeof(R) == 8;   // f64 ray on the f32 tree: widened intervals
    StealSlots<R> slots(steal_area);
    uint8_t* __restrict__ rv = steal_area + kStealSlotBytes<R>;
    int32_t* __restrict__ stk = stk_wave + lane;
    float ix, iy, iz, oix, oiy, oiz, slack, tbw;
    auto setup = [&]() {
        ix = inv_((float)T.d.x);
        iy = inv_((float)T.d.y);
        iz = inv_((float)T.d.z);
        oix = (float)T.o.x * ix;
        oiy = (float)T.o.y * iy;
        oiz = (float)T.o.z * iz;
        slack = kWide ? 0x1p-20f * fmaxf(fmaxf(fabsf(oix), fabsf(oiy)), fmaxf(fabsf(oiz), 0.0f)) : 0.0f;
    };
    auto bound = [&]() { tbw = kWide ? cull_bound(T.bound()) : 0.0f; };
    setup();
    bound();
    auto slab = [](float b, float i, float oi) {
        if constexpr (kWide) return __builtin_fmaf(b, i, -oi);
        else return b * i - oi;
    };
    const BvhNode<float>* __restrict__ nodes = cull_nodes(sc);
    int32_t sp = 0, sb = 0;             // stack entries [sb, sp): below sb they were given away
    int32_t owner = (int32_t)lane;      // the lane whose ray this lane traverses
    int32_t node = skip ? kDone : 0;
    int32_t leaf = 0;
    slots.init(lane, T);
    for (;;) {
        for (;;) {
            if (node < 0 && leaf == 0) {   // park the leaf, continue with the stack
                leaf = node;
                node = sp > sb ? stk[--sp * 64] : kDone;
            }
            const bool idle = node == kDone && leaf == 0, donor = sp > sb;
            const uint64_t mi = __ballot(idle), md = __ballot(donor);
            if (mi != 0 && md != 0) {
                const uint32_t np = min(__popcll(mi), __popcll(md));
                const uint32_t ri = __builtin_amdgcn_mbcnt_hi((uint32_t)(mi >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mi, 0u));
                const uint32_t rd = __builtin_amdgcn_mbcnt_hi((uint32_t)(md >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)md, 0u));
                const bool thief = idle && ri < np, give = donor && rd < np;
                if (give) rv[rd] = (uint8_t)lane;
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                const int32_t src = thief ? (int32_t)rv[ri] : (int32_t)lane;
                slots.fold(thief, owner, T, false);   // the thief's finished traversal
#if RTW_STEAL_TOP
                // the donor's top entry: its nearest postponed subtree
                const int32_t v_owner = bperm_i(owner, src), v_sb = bperm_i(sp, src) - 1;
#else
                const int32_t v_owner = bperm_i(owner, src), v_sb = bperm_i(sb, src);
#endif
                // every lane reads the ray of `src`: a thief its donor's, the
                // others their own (src = lane), so no copy of T is needed
                T.take(src);
                if (thief) {
                    owner = v_owner;
                    node = stk_wave[v_sb * 64 + src];
                    sp = sb = 0;
                    setup();
                }
                slots.refresh(thief, owner, T);       // the freshest shared bound
                if (thief) bound();
#if RTW_STEAL_TOP
                if (give) --sp;
#else
                if (give) ++sb;
#endif
            }
            const bool inner = node >= 0 && node != kDone;
            if (!__any(inner) || __all(leaf != 0 || node == kDone)) break;
            if (inner) {
                RTW_PROBE_LANES(1);
                ++nvis;
                const BvhNode<float>& nd = nodes[node];
                const float tb = kWide ? tbw : (float)T.bound();
                float tn[2], tf[2];
#pragma unroll
                for (int c = 0; c < 2; ++c) {
                    const float x0 = slab(nd.lo_x[c], ix, oix), x1 = slab(nd.hi_x[c], ix, oix);
                    const float y0 = slab(nd.lo_y[c], iy, oiy), y1 = slab(nd.hi_y[c], iy, oiy);
                    const float z0 = slab(nd.lo_z[c], iz, oiz), z1 = slab(nd.hi_z[c], iz, oiz);
                    tn[c] = fmaxf(fmaxf(fminf(x0, x1), fminf(y0, y1)), fmaxf(fminf(z0, z1), 0.0f));
                    tf[c] = fminf(fminf(fmaxf(x0, x1), fmaxf(y0, y1)), fminf(fmaxf(z0, z1), tb));
                    if constexpr (kWide) {
                        tn[c] = __builtin_fmaf(tn[c], 1.0f - 0x1p-20f, -slack);
                        tf[c] = __builtin_fmaf(tf[c], 1.0f + 0x1p-20f, slack);
                    }
                }
                const bool h0 = tn[0] <= tf[0], h1 = tn[1] <= tf[1];
                const int32_t c0 = nd.child[0], c1 = nd.child[1];
                if (h0 && h1) {
                    const bool first0 = tn[0] <= tn[1];
                    stk[sp * 64] = first0 ? c1 : c0;
                    ++sp;
                    node = first0 ? c0 : c1;
                } else if (h0 | h1) {
                    node = h0 ? c0 : c1;
                } else {
                    node = sp > sb ? stk[--sp * 64] : kDone;
                }
            }
        }
        if (!__any(leaf != 0)) break;   // no parked leaves: every lane is done
        const bool tested = leaf != 0;
        if (tested) {
            RTW_PROBE_LANES(2);
            test_leaf(sc, base, leaf, T, ntest);
            leaf = 0;
        }
        // share the bound: every lane on this ray culls with the best hit any
        // of them has found so far (f32: the exact key; f64: the bound only,
        // the exact (t, id) is folded when a lane leaves the ray)
        steal_share(slots, tested, owner, T);
        if (tested) bound();
    }
    slots.fold(true, owner, T, false);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    slots.result(lane, T);
}

// A ray with a NaN component hits nothing (every sphere, plane and light test
// compares a NaN), but its slab tests keep every box (fmin / fmax drop the
// NaN), so a traversal would visit the whole tree for a miss -- C5: the NaN
// directions a Lambertian point inside a light sphere samples (sphere.rs:
// 113-127) cost one wave a quarter of a second.  Such rays skip the traversal
// (bvh_dispatch: the trees outside LDS; a tree in LDS is small, its stealing
// traversal shares such a walk, and the check costs C2 more than it saves).
template <typename R>
__device__ __forceinline__ bool ray_nan(V3<R> o, V3<R> d) {
    return __builtin_isnan(o.x) | __builtin_isnan(o.y) | __builtin_isnan(o.z) | __builtin_isnan(d.x) |
           __builtin_isnan(d.y) | __builtin_isnan(d.z);
}

// `self` >= 0: the ray starts on that (isolated) sphere; it is tested first
// and, when the ray hits it again, that hit is the closest sphere hit (see
// isolated_spheres, host/bvh.hpp) and the traversal is skipped.
template <int kKind, typename R, typename TT>
__device__ __forceinline__ void bvh_dispatch(const DevScene<R>& sc, int32_t base, V3<R> o, V3<R> d,
                                             TT& T, int32_t* stk, uint32_t& nvis,
                                             uint32_t& ntest, int32_t self) {
    bool skip = ray_nan(o, d);
    if (!skip && self >= 0) {
        skip = T.test_hit(sc.sph[self], base + self);
        ++ntest;
    }
    if constexpr (kKind == kWorldBvh4) bvh4_traverse(sc, base, o, d, T, stk, nvis, ntest, skip);
    else if constexpr (kKind == kWorldBvhWW) bvh_traverse_ww(sc, base, o, d, T, stk, nvis, ntest, skip);
    else bvh_traverse(sc, base, o, d, T, stk, nvis, ntest, skip);
}

template <int kKind, bool kRobust>
__device__ __forceinline__ void bvh_closest(const DevScene<double>& sc, int32_t base, V3<double> o,
                                            V3<double> d, double tmin, double& tb, int32_t& best,
                                            int32_t* stk, uint32_t& nvis, uint32_t& ntest, int32_t self) {
    SphereTester<double, kRobust> T{o, d, tmin, tb, best};
    bvh_dispatch<kKind>(sc, base, o, d, T, stk, nvis, ntest, self);
    tb = T.tb;
    best = T.best;
}
template <int kKind, bool kRobust>
__device__ __forceinline__ void bvh_closest(const DevScene<float>& sc, int32_t base, V3<float> o,
                                            V3<float> d, float tmin, float& tb, int32_t& best,
                                            int32_t* stk, uint32_t& nvis, uint32_t& ntest, int32_t self) {
    SphereTester<float, kRobust> T;
    T.o = o;
    T.d = d;
    T.a = len2_f32(d);
    T.ia = __builtin_amdgcn_rcpf(T.a);
    T.tminb = __float_as_uint(tmin);
    T.ub = __float_as_uint(tb) - T.tminb;
    T.best = best;
    bvh_dispatch<kKind>(sc, base, o, d, T, stk, nvis, ntest, self);
    tb = T.bound();
    best = T.best;
}

// ---------------------------------------------------------------------------
// f64 hit points for the f32 kernels (kOptHit64).  The reference's t_min =
// f64::EPSILON (camera.rs:473) makes the bounce after a hit re-hit its own
// sphere ("acne") exactly when the rounded f64 hit point r.at(t) lies inside
// it -- a coin flip decided by f64 rounding that shapes the image (paths
// trapped inside spheres, NaN samples from Lambertian points inside light
// spheres).  f32 arithmetic flips that coin with other odds, so the f32 image
// drifts from the reference's region by region.  With kOptHit64 the f32
// kernel keeps the ray origin in f64 and computes, in f64 with the
// reference's operation order and no FMA contraction: the re-hit test of the
// sphere the ray starts on, the t of the sphere the f32 traversal picked, and
// the hit point o + d t.  Traversal, shading and sampling stay f32.
// ---------------------------------------------------------------------------
// Sphere::hit's roots, sphere.rs:61-80, with t in [EPSILON, inf] (f64, no FMA)
// on the sphere as given (DevScene::sph64: {c, radius})
__device__ __forceinline__ bool sphere_t_ref64(const R4<double>& S, V3<double> o, V3<double> d, double& t) {
#pragma clang fp contract(off)
    const double ocx = o.x - S.x, ocy = o.y - S.y, ocz = o.z - S.z, r = S.w;
    const double a = d.x * d.x + d.y * d.y + d.z * d.z;
    const double half_b = ocx * d.x + ocy * d.y + ocz * d.z;
    const double c = (ocx * ocx + ocy * ocy + ocz * ocz) - r * r;
    const double disc = half_b * half_b - a * c;
    if (!(disc > 0.0)) return false;
    const double sq = __builtin_sqrt(disc);
    double root = (-half_b - sq) / a;
    if (!(P<double>::kEps <= root && root <= (double)INFINITY)) {
        root = (-half_b + sq) / a;
        if (!(P<double>::kEps <= root && root <= (double)INFINITY)) return false;
    }
    t = root;
    return true;
}
// Plane::hit's t, plane.rs:64: -((o - p) . n) / (d . n) (f64, no FMA), on the
// plane as given (DevScene::pl64: {point, 0}, {normal, 0})
__device__ __forceinline__ double plane_t_ref64(const R4<double>* P, V3<double> o, V3<double> d) {
#pragma clang fp contract(off)
    const R4<double> pt = P[0], n = P[1];
    const double denom = d.x * n.x + d.y * n.y + d.z * n.z;
    return -(((o.x - pt.x) * n.x + (o.y - pt.y) * n.y + (o.z - pt.z) * n.z) / denom);
}
// Ray::at, o + d t (f64, no FMA)
__device__ __forceinline__ V3<double> ray_at64(V3<double> o, V3<double> d, double t) {
#pragma clang fp contract(off)
    return V3<double>{o.x + d.x * t, o.y + d.y * t, o.z + d.z * t};
}
__device__ __forceinline__ V3<double> to64(V3<float> v) { return V3<double>{v.x, v.y, v.z}; }
__device__ __forceinline__ V3<double> to64(V3<double> v) { return v; }
// An f32 direction as a GENERIC f64 value: the f32 value with pseudo-random
// bits below its 24-bit mantissa (a relative change < 2^-25: the same f32
// value).  The reference's directions are f64 results with rounding noise in
// every bit; a 24-bit value makes d.d exact and the products of d.(o - c)
// nearly so, which changes the odds of the ulp-level decisions above (the
// re-hit of a perfect mirror from inside, measured: tools/trace_paths.py).
// The bits come from a hash of the f32 bits (no RNG draw).
__device__ __forceinline__ uint32_t mix32(uint32_t h) {
    h ^= h >> 16;
    h *= 0x7feb352du;
    h ^= h >> 15;
    h *= 0x846ca68bu;
    h ^= h >> 16;
    return h;
}
__device__ __forceinline__ V3<double> dither64(V3<float> v) {
    RTW_PROBE_ABL_DITHER(v);
    const uint32_t h0 = mix32(__float_as_uint(v.x) ^ mix32(__float_as_uint(v.y) ^ mix32(__float_as_uint(v.z))));
    const uint32_t h1 = mix32(h0 + 0x9e3779b9u), h2 = mix32(h1 + 0x9e3779b9u);
    constexpr double kScale = 0x1p-25 / 4294967296.0;        // (h - 2^31) * 2^-57: |rel| < 2^-26
    return V3<double>{(double)v.x * (1.0 + ((double)h0 - 2147483648.0) * kScale),
                      (double)v.y * (1.0 + ((double)h1 - 2147483648.0) * kScale),
                      (double)v.z * (1.0 + ((double)h2 - 2147483648.0) * kScale)};
}

__device__ __forceinline__ V3<double> dither64(V3<double> v) { return v; }   // (R = double: unused)
template <typename R>
__device__ __forceinline__ V3<R> from64(V3<double> v) { return mk((R)v.x, (R)v.y, (R)v.z); }

// Vec3::normalize, self / self.length() (vec.rs), in f64, no FMA: the unit
// incoming direction both Metal and Dialectric start from (material.rs:414, 469)
__device__ __forceinline__ V3<double> unit64(V3<double> d) {
#pragma clang fp contract(off)
    const double l = __builtin_sqrt(d.x * d.x + d.y * d.y + d.z * d.z);
    return div3(d.x, d.y, d.z, l);
}
// Metal::scatter's direction (material.rs:407-421) in f64, no FMA, from the
// unit direction u: reflect(u, n) + us * fuzz, with reflect(v, n) = v - (n * 2)
// (v . n) (vec.rs); its dot with n decides absorption (returned in `keep`)
__device__ __forceinline__ V3<double> metal_dir64(V3<double> u, V3<double> n, double fuzz, V3<double> us,
                                                  bool& keep) {
#pragma clang fp contract(off)
    const double ux = u.x, uy = u.y, uz = u.z;
    const double vn = ux * n.x + uy * n.y + uz * n.z;
    const double rx = ux - (n.x * 2.0) * vn, ry = uy - (n.y * 2.0) * vn, rz = uz - (n.z * 2.0) * vn;
    const V3<double> out = {rx + us.x * fuzz, ry + us.y * fuzz, rz + us.z * fuzz};
    keep = out.x * n.x + out.y * n.y + out.z * n.z > 0.0;
    return out;
}
// Dialectric::scatter's direction (material.rs:458-487) in f64, no FMA, from
// the unit direction u and the material's f64 record M = {1/ior, r0 at 1/ior,
// r0 at ior, ior} (DevScene::mat64: the recip() and reflectance's r0 =
// ((1 - ratio) / (1 + ratio))^2 of both faces, computed once on the host with
// the same operations); the Open01 word is drawn only when refraction is
// possible (the || short circuit)
__device__ __forceinline__ V3<double> dielectric_dir64(V3<double> u, V3<double> n, bool front,
                                                       const R4<double>& M, Rng& g) {
#pragma clang fp contract(off)
    const double ratio = front ? M.x : M.w;
    const double ux = u.x, uy = u.y, uz = u.z;
    const double cos_t = __builtin_fmin(ux * -n.x + uy * -n.y + uz * -n.z, 1.0);
    const double sin_t = __builtin_sqrt(1.0 - cos_t * cos_t);
    bool refl = ratio * sin_t > 1.0;
    if (!refl) {
        const double r0 = front ? M.y : M.z;             // Dialectric::reflectance, powi(5) as LLVM expands it
        const double x = 1.0 - cos_t, x2 = x * x;
        refl = r0 + (1.0 - r0) * (x * (x2 * x2)) > P<double>::u_open01(g.next());
    }
    if (refl) {
        const double vn = ux * n.x + uy * n.y + uz * n.z;
        return V3<double>{ux - (n.x * 2.0) * vn, uy - (n.y * 2.0) * vn, uz - (n.z * 2.0) * vn};
    }
    // refract(v, n, eta), vec.rs: perp = (v + n cos) eta, par = n * -sqrt(1 - perp.perp)
    const double c2 = __builtin_fmin(ux * -n.x + uy * -n.y + uz * -n.z, 1.0);
    const double px = (ux + n.x * c2) * ratio, py = (uy + n.y * c2) * ratio, pz = (uz + n.z * c2) * ratio;
    const double q = -__builtin_sqrt(1.0 - (px * px + py * py + pz * pz));
    return V3<double>{px + n.x * q, py + n.y * q, pz + n.z * q};
}
// Metal::scatter and Dialectric::scatter for an f64 sphere hit (kOptHit64)
// in one pass: both start from the unit incoming direction u, its dot with
// the normal and the mirror direction (vec.rs reflect); Metal perturbs it by
// fuzz * UnitSphere (drawn first, as in the separate path), Dialectric keeps
// it on total internal reflection or a Schlick draw and refracts otherwise.
// The lanes of a wave that hit either material run it together.  Per lane
// the draws and operations are metal_dir64's / dielectric_dir64's:
// Dialectric's cos_theta = min(u . -n, 1) is min(-(u . n), 1) bit for bit
// (negation is exact and round-to-nearest symmetric).
// `kRefSphere`: Metal's UnitSphere by the reference's rejection loop in f64
// (the f64 parity kernels), else the f32 kernels' direct sampler carried into
// f64 (dither64).
#ifndef RTW_HIT64_LAMB64
#define RTW_HIT64_LAMB64 1   // hit64 Lambertian: the direction in f64 (r05 default; 0 = in f32)
#endif
#ifndef RTW_HIT64_TRIG32
// hit64 f64 Lambertian direction with the azimuth's sin / cos in f32 (experiment:
// -1.9 % time, but the f32 paths' statistics fall back to the f32 direction's --
// 2.793 segments per sample vs f64's 2.764, NaN pixels 15.0 % vs 14.7 %;
// profiles/r05_hit64_trig32_ab.jsonl)
#define RTW_HIT64_TRIG32 0
#endif
#ifndef RTW_HIT64_REF_SPHERE
#define RTW_HIT64_REF_SPHERE 0   // hit64 Metal: 1 = the reference's f64 rejection loop (experiment)
#endif
template <bool kRefSphere = false>
__device__ __forceinline__ V3<double> specular_dir64(bool metal, V3<double> d, V3<double> n, bool front,
                                                     const R4<double>& M, Rng& g, bool& keep) {
#pragma clang fp contract(off)
    V3<double> us = {0.0, 0.0, 0.0};
    if (metal) {
        if constexpr (kRefSphere) us = unit_sphere<double>(g);
        else us = dither64(unit_sphere<float>(g));
    }
    const V3<double> u = unit64(d);
    const double vn = u.x * n.x + u.y * n.y + u.z * n.z;
    const V3<double> r = {u.x - (n.x * 2.0) * vn, u.y - (n.y * 2.0) * vn, u.z - (n.z * 2.0) * vn};
    keep = true;
    if (metal) {
        const double fuzz = M.w;
        const V3<double> out = {r.x + us.x * fuzz, r.y + us.y * fuzz, r.z + us.z * fuzz};
        keep = out.x * n.x + out.y * n.y + out.z * n.z > 0.0;
        return out;
    }
    const double ratio = front ? M.x : M.w;
    const double cos_t = __builtin_fmin(-vn, 1.0);
    const double sin_t = __builtin_sqrt(1.0 - cos_t * cos_t);
    bool refl = ratio * sin_t > 1.0;
    if (!refl) {
        const double r0 = front ? M.y : M.z;   // Dialectric::reflectance, powi(5) as LLVM expands it
        const double x = 1.0 - cos_t, x2 = x * x;
        refl = r0 + (1.0 - r0) * (x * (x2 * x2)) > P<double>::u_open01(g.next());
    }
    if (refl) return r;
    // refract(v, n, eta), vec.rs: perp = (v + n cos) eta, par = n * -sqrt(1 - perp.perp)
    const double px = (u.x + n.x * cos_t) * ratio, py = (u.y + n.y * cos_t) * ratio, pz = (u.z + n.z * cos_t) * ratio;
    const double q = -__builtin_sqrt(1.0 - (px * px + py * py + pz * pz));
    return V3<double>{px + n.x * q, py + n.y * q, pz + n.z * q};
}
// the outward normal (p - c) / radius, sphere.rs:82-83 (f64, no FMA)
__device__ __forceinline__ V3<double> sphere_normal64(V3<double> p, const R4<double>& S) {
#pragma clang fp contract(off)
    return div3(p.x - S.x, p.y - S.y, p.z - S.z, S.w);
}
__device__ __forceinline__ bool front64(V3<double> d, V3<double> n) {
#pragma clang fp contract(off)
    return d.x * n.x + d.y * n.y + d.z * n.z < 0.0;
}

// The f32 sphere test with one sphere id excluded (kOptHit64: the sphere the
// ray starts on, whose re-hit is decided in f64).
template <bool kRobust>
struct SphereTesterX : SphereTester<float, kRobust> {
    int32_t excl;
    __device__ __forceinline__ void take(int32_t src) {
        SphereTester<float, kRobust>::take(src);
        excl = bperm_i(excl, src);
    }
    __device__ __forceinline__ void test(const R4<float>& s, int32_t id) {
        const uint32_t u = sphere_u<kRobust>(s, this->o, this->d, this->a, this->ia, this->tminb);
        const bool upd = (u < this->ub || (u == this->ub && id < this->best)) && id != excl;
        this->ub = upd ? u : this->ub;
        this->best = upd ? id : this->best;
    }
};
template <int kKind, bool kRobust>
__device__ __forceinline__ void bvh_closest_excl(const DevScene<float>& sc, int32_t base, V3<float> o,
                                                 V3<float> d, float tmin, float& tb, int32_t& best,
                                                 int32_t* stk, uint32_t& nvis, uint32_t& ntest, int32_t excl) {
    SphereTesterX<kRobust> T;
    T.o = o;
    T.d = d;
    T.a = len2_f32(d);
    T.ia = __builtin_amdgcn_rcpf(T.a);
    T.tminb = __float_as_uint(tmin);
    T.ub = __float_as_uint(tb) - T.tminb;
    T.best = best;
    T.excl = excl;
    bvh_dispatch<kKind>(sc, base, o, d, T, stk, nvis, ntest, -1);
    tb = T.bound();
    best = T.best;
}

// The same two queries with subtree stealing (while-while kernels): every
// active lane of the wave calls them -- a lane whose ray needs no traversal
// (the own-sphere shortcut: `skip`) helps the others.
template <bool kRobust>
__device__ __forceinline__ void bvh_closest_steal(const DevScene<double>& sc, int32_t base, V3<double> o,
                                                  V3<double> d, double tmin, double& tb, int32_t& best,
                                                  int32_t* stk_wave, uint32_t lane, unsigned char* steal_area,
                                                  uint32_t& nvis, uint32_t& ntest, int32_t self) {
    SphereTester<double, kRobust> T{o, d, tmin, tb, best};
    bool skip = false;
    if (self >= 0) {
        skip = T.test_hit(sc.sph[self], base + self);
        ++ntest;
    }
    bvh_traverse_steal(sc, base, T, stk_wave, lane, steal_area, nvis, ntest, skip);
    tb = T.tb;
    best = T.best;
}
template <bool kRobust>
__device__ __forceinline__ void bvh_closest_steal(const DevScene<float>& sc, int32_t base, V3<float> o, V3<float> d,
                                                  float tmin, float& tb, int32_t& best, int32_t* stk_wave,
                                                  uint32_t lane, unsigned char* steal_area, uint32_t& nvis,
                                                  uint32_t& ntest, int32_t self) {
    SphereTester<float, kRobust> T;
    T.o = o;
    T.d = d;
    T.a = len2_f32(d);
    T.ia = __builtin_amdgcn_rcpf(T.a);
    T.tminb = __float_as_uint(tmin);
    T.ub = __float_as_uint(tb) - T.tminb;
    T.best = best;
    bool skip = false;
    if (self >= 0) {
        skip = T.test_hit(sc.sph[self], base + self);
        ++ntest;
    }
    bvh_traverse_steal(sc, base, T, stk_wave, lane, steal_area, nvis, ntest, skip);
    tb = T.bound();
    best = T.best;
}
template <bool kRobust>
__device__ __forceinline__ void bvh_closest_excl_steal(const DevScene<float>& sc, int32_t base, V3<float> o,
                                                       V3<float> d, float tmin, float& tb, int32_t& best,
                                                       int32_t* stk_wave, uint32_t lane, unsigned char* steal_area,
                                                       uint32_t& nvis, uint32_t& ntest, int32_t excl, bool skip) {
    SphereTesterX<kRobust> T;
    T.o = o;
    T.d = d;
    T.a = len2_f32(d);
    T.ia = __builtin_amdgcn_rcpf(T.a);
    T.tminb = __float_as_uint(tmin);
    T.ub = __float_as_uint(tb) - T.tminb;
    T.best = best;
    T.excl = excl;
    bvh_traverse_steal(sc, base, T, stk_wave, lane, steal_area, nvis, ntest, skip);
    tb = T.bound();
    best = T.best;
}

// Light pdf through the light BVH (KParams::light_bvh): every light sphere the
// ray (o, d) hits with t in [0, inf] contributes its solid-angle pdf
// (HittableList::pdf_value, hittable_list.rs:408-412; sphere.rs:101-111).
// Boxes only cull.  The traversal reuses the lane's LDS stack.
//
// Both children of a node are slab-tested against [0, inf); the visit order
// does not matter for an all-hits query.
// Light-pdf work of one lane, counted into KParams::counters[7] / [8]: light
// tests (every light of the big list, a visited grid cell or a light-BVH leaf
// that the ray is tested against) and light-grid cells visited.
struct LightWork {
    uint32_t tests = 0, cells = 0;
};
// ... added to the wave's u64 counters in LDS (w[0] tests, w[1] cells): from
// any subset of lanes (LDS atomics), or from the whole converged wave (one sum)
__device__ __forceinline__ void light_work_lane(unsigned long long* w, const LightWork& lw) {
    if (lw.tests) atomicAdd(w, (unsigned long long)lw.tests);
    if (lw.cells) atomicAdd(w + 1, (unsigned long long)lw.cells);
}
__device__ __forceinline__ void light_work_wave(unsigned long long* w, LightWork lw, uint32_t lane) {
    uint32_t t = lw.tests, c = lw.cells;
    for (int off = 32; off > 0; off >>= 1) {
        t += (uint32_t)__shfl_xor((int)t, off);
        c += (uint32_t)__shfl_xor((int)c, off);
    }
    if (lane == 0) {
        w[0] += t;
        w[1] += c;
    }
}

template <typename R, typename Leaf>
__device__ __forceinline__ void light_bvh_walk(const DevScene<R>& sc, V3<R> o, V3<R> d,
                                               int32_t* __restrict__ stk, Leaf&& leaf) {
    const R ix = inv_(d.x), iy = inv_(d.y), iz = inv_(d.z);
    const R oix = o.x * ix, oiy = o.y * iy, oiz = o.z * iz;
    int32_t sp = 0;
    int32_t node = 0;
    for (;;) {
        if (node >= 0) {
            const BvhNode<R>& nd = sc.lbvh[node];
            bool h[2];
#pragma unroll
            for (int c = 0; c < 2; ++c) {
                const R x0 = nd.lo_x[c] * ix - oix, x1 = nd.hi_x[c] * ix - oix;
                const R y0 = nd.lo_y[c] * iy - oiy, y1 = nd.hi_y[c] * iy - oiy;
                const R z0 = nd.lo_z[c] * iz - oiz, z1 = nd.hi_z[c] * iz - oiz;
                const R tn = fmax(fmax(fmin(x0, x1), fmin(y0, y1)), fmax(fmin(z0, z1), (R)0));
                const R tf = fmin(fmax(x0, x1), fmin(fmax(y0, y1), fmax(z0, z1)));
                h[c] = tn <= tf;
            }
            const int32_t c0 = nd.child[0], c1 = nd.child[1];
            if (h[0] && h[1]) {
                stk[sp * 64] = c1;
                ++sp;
                node = c0;
                continue;
            }
            if (h[0] | h[1]) {
                node = h[0] ? c0 : c1;
                continue;
            }
        } else {
            const uint32_t code = (uint32_t)~node;
            const uint32_t first = code >> 4, cnt = code & 15u;
            for (uint32_t k = 0; k < cnt; ++k) leaf(first + k);
        }
        if (sp == 0) break;
        --sp;
        node = stk[sp * 64];
    }
}

// f32: light_hit_f32 / light_pdf_f32 as in lights_pdf_sum; pdfs summed in walk order.
template <bool kRobust>
__device__ __forceinline__ float lights_pdf_bvh(const DevScene<float>& sc, V3<float> o, V3<float> d,
                                                int32_t* __restrict__ stk, LightWork& lw) {
    const float a = len2_f32(d);
    const float ia = __builtin_amdgcn_rcpf(a);
    float acc = 0.f;
    light_bvh_walk(sc, o, d, stk, [&](uint32_t k) {
        ++lw.tests;
        const R4<float> L = sc.lsph[k];
        const bool hit = light_hit_f32<kRobust>(L, o, d, a, ia);
        if (hit) acc += light_pdf_f32(L, o);
    });
    return acc;
}
// f64 (parity mode): collect the hit lights' list indices, then sum their
// pdfs in LIST order with the reference arithmetic -- bit-identical to the
// linear sum (misses add +0.0, which changes nothing).  More than 8 hits
// falls back to the linear loop.
template <bool kRobust>
__device__ __forceinline__ double lights_pdf_bvh(const DevScene<double>& sc, V3<double> o, V3<double> d,
                                                 int32_t* __restrict__ stk, LightWork& lw) {
    const LightPre pre(o, d);
    return lights_sum_in_list_order(sc.lights, o, d, [&](auto&& add) {
        light_bvh_walk(sc, o, d, stk, [&](uint32_t k) {
            ++lw.tests;
            const R4<double> L = sc.lsph[k];
            double t;
            if (pre.may_hit(L) && sphere_t(mk(L.x, L.y, L.z), L.w * L.w, o, d, 0.0, t)) add(sc.lid[k]);
        });
    });
}

// f32: the big list, then the walk; a light counts in the cell whose interval
// holds its closest-approach parameter tc = -(d . (o - c)) / (d . d)
template <bool kRobust>
__device__ __forceinline__ float lights_pdf_grid(const DevScene<float>& sc, V3<float> o, V3<float> d,
                                                 LightWork& lw) {
    const float a = len2_f32(d);
    const float ia = __builtin_amdgcn_rcpf(a);
    float acc = 0.f;
    lw.tests += sc.lg_big;
    for (uint32_t k = 0; k < sc.lg_big; ++k) {
        const R4<float> L = sc.lg_sph[k];
        if (light_hit_f32<kRobust>(L, o, d, a, ia)) acc += light_pdf_f32(L, o);
    }
    light_grid_walk(sc, o, d, [&](uint32_t k, float te, float tx) {
        ++lw.tests;
        const R4<float> L = sc.lg_sph[k];
        const float fx = o.x - L.x, fy = o.y - L.y, fz = o.z - L.z;
        const float tc = -__builtin_fmaf(d.z, fz, __builtin_fmaf(d.y, fy, d.x * fx)) * ia;
        if (light_hit_f32<kRobust>(L, o, d, a, ia) & (tc >= te) & (tc < tx)) acc += light_pdf_f32(L, o);
    }, &lw.cells);
    return acc;
}
// lights_pdf_grid by the whole wave (f32, KParams::grid_piece = P > 0).  A ray
// that skims a flat light layer walks the grid's whole width (C5: a ground
// point sampling one of 50k lights at the same height, ~150 cells of ~4 lights
// each) while most rays walk a few cells, and a lane-per-ray walk keeps its
// wave for the longest one (C5: 10 % of lanes active).  Here every lane of
// the wave walks for the pending rays (`pend`; the ray is (o, d)): each ray's
// grid interval [tn, tf] is cut into k = ceil(cells / P) pieces of equal
// length in t, the pieces of all rays are dealt to the 64 lanes round by
// round, every piece's pdf sum lands in an LDS slot, and each ray's owner
// adds its pieces up in order.  The cut depends on the ray and P alone and
// the sum runs in piece order, so the result does not depend on which rays
// share the wave; the first piece starts from the big list's sum, so a
// one-piece ray (most of them) sums exactly as lights_pdf_grid.  `slots`:
// `cap` (a multiple of 64) floats of the wave's LDS; every lane of the wave
// calls this (converged), with wave-uniform P.
template <bool kRobust, typename Mark>
__device__ __forceinline__ float lights_pdf_grid_coop(const DevScene<float>& sc, bool pend, V3<float> o, V3<float> d,
                                                   uint32_t P, float* __restrict__ slots, uint32_t cap,
                                                   uint32_t lane, LightWork& lw, Mark&& mark) {
    float acc = 0.f, tn = 0.f, tf = 0.f;
    uint32_t k = 0;
    if (pend) {
        const float a = len2_f32(d);
        const float ia = __builtin_amdgcn_rcpf(a);
        lw.tests += sc.lg_big;
        for (uint32_t q = 0; q < sc.lg_big; ++q) {
            const R4<float> L = sc.lg_sph[q];
            if (light_hit_f32<kRobust>(L, o, d, a, ia)) acc += light_pdf_f32(L, o);
        }
        uint32_t cells = 0;
        if (light_grid_span(sc, o, d, grid_inv(d.x), grid_inv(d.y), grid_inv(d.z), tn, tf, cells))
            k = (cells + P - 1u) / P;
    }
    // first piece of each ray: exclusive prefix of k over the lanes
    uint32_t incl = k;
#pragma unroll
    for (uint32_t off = 1; off < 64; off <<= 1) {
        const uint32_t v = (uint32_t)__shfl_up((int)incl, off);
        if (lane >= off) incl += v;
    }
    const uint32_t first = incl - k, total = (uint32_t)__shfl((int)incl, 63);
    mark(13);
    for (uint32_t b = 0; b < total; b += cap) {
        const uint32_t e = min(b + cap, total);
        for (uint32_t r = b; r < e; r += 64) {
            const uint32_t g = r + lane;
            // the piece's ray: the last lane whose first piece is <= g
            uint32_t own = 0;
#pragma unroll
            for (uint32_t step = 32; step; step >>= 1) {
                const uint32_t f = (uint32_t)__shfl((int)first, (int)(own + step));
                own = f <= g ? own + step : own;
            }
            const V3<float> ro = mk(bperm_f(o.x, own), bperm_f(o.y, own), bperm_f(o.z, own));
            const V3<float> rd = mk(bperm_f(d.x, own), bperm_f(d.y, own), bperm_f(d.z, own));
            const float rtn = bperm_f(tn, own), rtf = bperm_f(tf, own), racc = bperm_f(acc, own);
            const uint32_t rk = (uint32_t)bperm_i((int32_t)k, own), rfirst = (uint32_t)bperm_i((int32_t)first, own);
            if (g < e) {
                const uint32_t j = g - rfirst;
                const float step = (rtf - rtn) / (float)rk;
                auto t_at = [&](uint32_t q) { return q == 0 ? rtn : __builtin_fmaf((float)q, step, rtn); };
                const float ra = len2_f32(rd);
                const float ria = __builtin_amdgcn_rcpf(ra);
                float part = j == 0 ? racc : 0.f;
                auto test = [&](const R4<float>& L, float te, float tx) {
                    const float fx = ro.x - L.x, fy = ro.y - L.y, fz = ro.z - L.z;
                    const float tc = -__builtin_fmaf(rd.z, fz, __builtin_fmaf(rd.y, fy, rd.x * fx)) * ria;
                    if (light_hit_f32<kRobust>(L, ro, rd, ra, ria) & (tc >= te) & (tc < tx))
                        part += light_pdf_f32(L, ro);
                };
#if RTW_GRID_REC
                RTW_PROBE_LANES(11);
                light_grid_walk_piece_rec(sc, sc.lg_rec, sc.lg_sph, ro, rd, grid_inv(rd.x), grid_inv(rd.y),
                                          grid_inv(rd.z), t_at(j), t_at(j + 1), j == 0, j + 1 == rk,
                                          [&](const R4<float>& L, auto&&, float te, float tx) {
                                              RTW_PROBE_LANES(12);
                                              test(L, te, tx);
                                          }, &lw.cells, &lw.tests);
#else
                light_grid_walk_piece(sc, ro, rd, grid_inv(rd.x), grid_inv(rd.y), grid_inv(rd.z), t_at(j),
                                      t_at(j + 1), j == 0, j + 1 == rk, [&](uint32_t q, float te, float tx) {
                    ++lw.tests;
                    test(sc.lg_sph[q], te, tx);
                }, &lw.cells);
#endif
                slots[g - b] = part;
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        mark(14);
        if (k) {
            const uint32_t g0 = max(first, b), g1 = min(first + k, e);
            for (uint32_t g = g0; g < g1; ++g) acc = g == first ? slots[g - b] : acc + slots[g - b];
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        mark(15);
    }
    return acc;
}

// f64 (parity mode): the hit lights' list indices, summed in LIST order
// (lights_sum_in_list_order) as in lights_pdf_bvh.
template <bool kRobust>
__device__ __forceinline__ double lights_pdf_grid(const DevScene<double>& sc, V3<double> o, V3<double> d,
                                                  LightWork& lw) {
    const LightPre pre(o, d);   // the f32 pre-pass rules out the lights the ray misses
    const double ia = 1.0 / (d.x * d.x + d.y * d.y + d.z * d.z);
    return lights_sum_in_list_order(sc.lights, o, d, [&](auto&& add) {
        lw.tests += sc.lg_big;
        for (uint32_t k = 0; k < sc.lg_big; ++k) {
            const R4<double> L = sc.lg_sph[k];
            double t;
            if (pre.may_hit(L) && sphere_t(mk(L.x, L.y, L.z), L.w * L.w, o, d, 0.0, t)) add(sc.lg_id[k]);
        }
        light_grid_walk(sc, o, d, [&](uint32_t k, double te, double tx) {
            ++lw.tests;
            const R4<double> L = sc.lg_sph[k];
            double t;
            if (pre.may_hit(L) && sphere_t(mk(L.x, L.y, L.z), L.w * L.w, o, d, 0.0, t)) {
                const double tc = -((o.x - L.x) * d.x + (o.y - L.y) * d.y + (o.z - L.z) * d.z) * ia;
                if (tc >= te && tc < tx) add(sc.lg_id[k]);
            }
        }, &lw.cells);
    });
}

// lights_pdf_grid (f64) by the whole wave.  The sum needs the SET of lights
// the f64 test hits, summed in LIST order; which structure finds them is free.
// So the walk runs in f32 -- the f32 kernels' piece cut (lights_pdf_grid_coop:
// each pending ray's grid interval cut into k = ceil(cells / P) pieces of
// equal length in t, dealt to the 64 lanes), on the f32 copy of the grid
// (DevScene::lg_sph32 and the grid box rounded to f32) -- and a light of a
// visited cell is a candidate when the f64 path's f32 pre-pass (LightPre /
// light_may_hit: slack far above the f32 error) says the ray may hit it and
// its f32 closest-approach parameter falls in the cell's interval: every light
// the f64 test hits is a candidate exactly once (the intervals partition the
// line; the host pads the cells' lists beyond the f32 rounding).  The owner
// sums Sphere::pdf_value over its candidates in list order, in f64 (a
// candidate the f64 test misses adds +0.0: no bit changes).  In passes over
// list indices >= lo: a piece keeps the kPieceIds smallest candidate indices
// >= lo it finds, sorted, in its LDS slot ([count, ids]); each owner merges
// its pieces' indices and the big list's into its kMax smallest; every index
// up to `bound` -- the largest kept index of a piece or an owner list that
// had to drop some, else unbounded -- is then known, so the owner sums those
// and, when something was dropped, the wave walks again for its rays with
// lo = bound + 1 (each pass sums at least one index: the walk always ends).
// Bit-identical to lights_pdf_grid and the linear list-order sum.  (Round 4
// walked in f64 -- f64 DDA, f64 records, the f64 test in the piece: C3 / C5
// spilled the path state at every trip.)  Every lane of the wave calls this
// (converged), with wave-uniform P; `cap_words` (a multiple of 64) of LDS at
// `slots`.
// The pending f64 ray (o, d) is read from the wave's LDS stash (`ray`: words
// [(2k) 64 + lane], [(2k + 1) 64 + lane] for k = 0..5, the kernel's layout)
// where it is needed -- the f32 ray at the start of a pass, the pdfs at its
// end -- so it is not held in registers across the walk's rounds.
// The light grid of an f64 scene as the f32 walk reads it: the arrays, and
// the grid box, cells and their counts rounded to f32.
struct Grid64 {
    const uint32_t* lg_start;
    const R4<float>* lg_rec;          // the cell records (f32 lights: lg_sph32's values)
    const R4<float>* lg_sph32;        // DevScene<double>::lg_sph32
    const uint32_t* lg_id;
    const R4<double>* lights;         // the light list (f64 records: the pdfs)
    float lo[3], hi[3], cell[3], inv[3];
    uint32_t n[3], big;
};
// The cooperative walk with the list-order sum, both precisions (R: the sum).
// `g`: the grid as the f32 walk reads it (lg_start, lg_sph, box, cells);
// `rec` its cell records, `lg_id` the items' list indices, `big` the big
// list's length; (of, df) the pending ray in f32 and ia_own = 1 / (df . df)
// as the owner's tests compute it.  cand(L, ro, rd, ra, ria, ron, rdn): may
// the ray hit light L (a piece's test; the owner's ray bperm'd, ra = its
// len2_f32, ron / rdn = |o|_1, |d|_1); big_hit(L): the owner's test of a big
// light; sum_ids(ids, n, bound, acc): acc += the pdfs of ids[0..n) up to
// `bound`, in that (list) order; pdf_at(id, owner): light id's pdf for the ray
// of lane `owner` (RTW_COOP_DEAL: evaluated by any lane).  `mark(id)`: the clock probes' section marks
// (RTW_CLOCK builds; else a no-op).
template <typename R, typename Cand, typename BigHit, typename SumIds, typename PdfAt, typename Mark>
__device__ __forceinline__ R lights_pdf_grid_coop_list(const DevScene<float>& g, const R4<float>* __restrict__ rec,
                                                       const uint32_t* __restrict__ lg_id, uint32_t big, V3<float> of,
                                                       V3<float> df, float ia_own, bool pend, uint32_t P,
                                                       uint32_t* __restrict__ slots, uint32_t cap_words, uint32_t lane,
                                                       LightWork& lw, Cand&& cand, BigHit&& big_hit, SumIds&& sum_ids,
                                                       PdfAt&& pdf_at, Mark&& mark) {
    // a piece's slot: [count, ids...] padded to 8 words (the owner reads it as two
    // 16-byte LDS loads)
    constexpr uint32_t kPieceIds = kCoop64PieceIds, kSlot = kCoop64Slot, kMax = RTW_COOP64_MAX;
    const uint32_t cap = cap_words / (kSlot * 64) * 64;   // pieces per round
    // (the host sizes the stack area for at least one round of 64 pieces, so a
    // smaller area is a host error: every pending ray ends NaN, never a loop
    // that cannot advance)
    if (cap == 0) return pend ? (R)NAN : (R)0;
    float tn = 0.f, tf = 0.f;
    uint32_t k = 0, cells = 0;
    const bool walks = pend && light_grid_span(g, of, df, grid_inv(df.x), grid_inv(df.y), grid_inv(df.z), tn, tf, cells);
    // pieces of Q cells (wave-uniform): the sum does not depend on the cut (list
    // order), so the wave's pending cells are spread over its lanes -- one round
    // of at most 64 pieces (sum ceil(c / Q) <= C / Q + n <= 64) unless that needs
    // pieces longer than P, the longest the tuning allows (C3: ~27 short rays per
    // trip walked as ~27 one-piece rays left most lanes idle)
    uint32_t Q = P;
    if constexpr (RTW_COOP_ADAPT != 0) {
        uint32_t C = walks ? cells : 0u;
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) C += (uint32_t)__shfl_xor((int)C, off);
        const uint32_t nr = (uint32_t)__popcll(__ballot(walks));
        if (nr < 64u) Q = min(P, max(kCoopAdaptMin, (C + (63u - nr)) / (64u - nr)));
    }
    // at most `cap` pieces (longer pieces for a longer ray): every ray's
    // pieces fit one round, so its owner finds all of them in the slots
    if (walks) k = min((cells + Q - 1u) / Q, cap);
    const uint32_t ia_bits = __float_as_uint(ia_own);
    // the big list's candidates of the pending ray: tested once per walk, not at
    // each of the owner's merges (their loads were on the merge's critical path)
    constexpr uint32_t kBigC = 2;
    uint32_t bigc[kBigC] = {0u, 0u};
    uint32_t nbig = 0;
    bool big_over = false;
    if (pend && big) {
        lw.tests += big;
        for (uint32_t q = 0; q < big; ++q) {
            if (big_hit(g.lg_sph[q])) {
                if (nbig < kBigC) bigc[nbig++] = lg_id[q];
                else big_over = true;
            }
        }
    }
    R acc = (R)0;
    uint32_t lo = 0;
    bool more = pend;           // the ray still needs a walk (over list indices >= lo)
    while (__any(more)) {
        const uint32_t kp = more ? k : 0u;   // this walk's pieces
        uint32_t incl = kp;
#pragma unroll
        for (uint32_t off = 1; off < 64; off <<= 1) {
            const uint32_t v = (uint32_t)__shfl_up((int)incl, off);
            if (lane >= off) incl += v;
        }
        const uint32_t first = incl - kp, total = (uint32_t)__shfl((int)incl, 63);
        bool walk_again = false;
        mark(13);
        // rounds of whole rays: [B, Bn) holds the pieces of the rays that start
        // at B or later and end by B + cap (a pending ray without pieces -- it
        // misses the grid -- sums its big-list candidates in the first round)
        for (uint32_t B = 0;;) {
            const bool mine = more && (kp ? first >= B && first + kp <= B + cap : B == 0);   // the ray is in the round
            const uint64_t later = __ballot(kp && first >= B && !mine);
            const uint32_t Bn = later ? (uint32_t)__shfl((int)first, (int)__builtin_ctzll(later)) : total;
            // a round of at most 64 pieces (the usual case: cap is 64 at the
            // host's minimum stack) keeps the mask of its pieces that hold a
            // candidate, so that an owner's merge reads only those slots
            const bool one_pass = RTW_COOP_HELD && Bn - B <= 64u;
            uint64_t held = ~0ull;
            for (uint32_t r = B; r < Bn; r += 64) {
                const uint32_t gi = r + lane;
                bool has = false;
                uint32_t own = 0;
#pragma unroll
                for (uint32_t step = 32; step; step >>= 1) {
                    const uint32_t f = (uint32_t)__shfl((int)first, (int)(own + step));
                    own = f <= gi ? own + step : own;
                }
                const V3<float> ro = mk(bperm_f(of.x, own), bperm_f(of.y, own), bperm_f(of.z, own));
                const V3<float> rd = mk(bperm_f(df.x, own), bperm_f(df.y, own), bperm_f(df.z, own));
                const float rtn = bperm_f(tn, own), rtf = bperm_f(tf, own);
                const uint32_t rk = (uint32_t)bperm_i((int32_t)kp, own), rfirst = (uint32_t)bperm_i((int32_t)first, own);
                const uint32_t rlo = (uint32_t)bperm_i((int32_t)lo, own);
                const float ria = __uint_as_float((uint32_t)bperm_i((int32_t)ia_bits, own));
                if (gi < Bn) {
                    const uint32_t j = gi - rfirst;
                    const float step = (rtf - rtn) / (float)rk;
                    auto t_at = [&](uint32_t q) { return q == 0 ? rtn : __builtin_fmaf((float)q, step, rtn); };
                    // the owner's test quantities, from the same f32 ray
                    const float ron = fabsf(ro.x) + fabsf(ro.y) + fabsf(ro.z), rdn = fabsf(rd.x) + fabsf(rd.y) + fabsf(rd.z);
                    const float ra = len2_f32(rd);
                    uint32_t* ent = slots + (gi - B) * kSlot + 1;
                    uint32_t cnt = 0;
#if RTW_PIECE_REG
                    // (RTW_PIECE_REG: the candidates in registers, the slot written once)
                    uint32_t pid[kPieceIds];
#pragma unroll
                    for (uint32_t q = 0; q < kPieceIds; ++q) pid[q] = 0xffffffffu;
#endif
                    // a light of the piece: a candidate (its list index kept) when the
                    // test may hit it in the cell's interval; idx(): its lg_id slot
                    auto test = [&](const R4<float>& L, auto&& idx, float te, float tx) {
                        if (cand(L, ro, rd, ra, ria, ron, rdn)) {
                            const float tc = -__builtin_fmaf(rd.z, ro.z - L.z, __builtin_fmaf(rd.y, ro.y - L.y,
                                                                                               rd.x * (ro.x - L.x))) * ria;
                            if (!(tc >= te && tc < tx)) return;
                            const uint32_t id = lg_id[idx()];
                            if (id >= rlo) {
                                // the piece's kPieceIds smallest, sorted (rare: a candidate)
#if RTW_PIECE_REG
                                ++cnt;
                                (void)sorted_insert(pid, id);
                                return;
#endif
                                uint32_t m = min(cnt, kPieceIds);
                                ++cnt;
                                if (m == kPieceIds) {
                                    if (id > ent[kPieceIds - 1]) return;
                                    --m;                               // the largest gives way
                                }
                                while (m > 0 && ent[m - 1] > id) {
                                    ent[m] = ent[m - 1];
                                    --m;
                                }
                                ent[m] = id;
                            }
                        }
                    };
#if RTW_GRID_REC
                    light_grid_walk_piece_rec(g, rec, g.lg_sph, ro, rd, grid_inv(rd.x), grid_inv(rd.y),
                                              grid_inv(rd.z), t_at(j), t_at(j + 1), j == 0, j + 1 == rk, test,
                                              &lw.cells, &lw.tests);
#else
                    light_grid_walk_piece(g, ro, rd, grid_inv(rd.x), grid_inv(rd.y), grid_inv(rd.z), t_at(j),
                                          t_at(j + 1), j == 0, j + 1 == rk, [&](uint32_t q, float te, float tx) {
                        ++lw.tests;
                        test(g.lg_sph[q], [q]() { return q; }, te, tx);
                    }, &lw.cells);
#endif
#if RTW_PIECE_REG
                    {
                        typedef uint32_t u4 __attribute__((ext_vector_type(4)));
                        static_assert(kPieceIds <= 7 && kSlot == 8, "the slot as two 16-byte stores");
                        uint32_t w[7];
#pragma unroll
                        for (uint32_t q = 0; q < 7; ++q) w[q] = q < kPieceIds ? pid[q < kPieceIds ? q : 0] : 0xffffffffu;
                        u4* sl = reinterpret_cast<u4*>(ent - 1);
                        sl[0] = u4{cnt, w[0], w[1], w[2]};
                        sl[1] = u4{w[3], w[4], w[5], w[6]};
                    }
#else
                    ent[-1] = cnt;
#endif
                    has = cnt != 0;
                }
                const uint64_t h = __ballot(has);
                if (one_pass) held = h;
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            mark(14);
            // every candidate >= lo of this ray is in its pieces' slots (and the
            // big list) unless a piece kept only its kPieceIds smallest: its owner
            // merges the kMax smallest, sums them in list order, and merges again
            // above the last one summed until done -- or until a piece's dropped
            // candidates are needed, which takes another walk.  RTW_COOP_DEAL: the
            // owners' merges run together and the pdfs of all their summable ids
            // are dealt to the wave's lanes (pdf_at(id, owner): any lane evaluates
            // a candidate for the owner's ray); each owner then adds its values
            // in list order, fetched by ds_bpermute -- the sum of each ray is the
            // same, its pdfs no longer computed by its owner lane alone
            bool owning = mine;
            while (RTW_COOP_DEAL ? __any(owning) : owning) {
                uint32_t ids[kMax];
#pragma unroll
                for (uint32_t q = 0; q < kMax; ++q) ids[q] = 0xffffffffu;
                uint32_t n = 0, bp = 0xffffffffu, bound = 0xffffffffu;   // bp: below a piece's dropped candidates
                if (owning) {
                    RTW_PROBE_LANES(13);
                    bool dropped = false;
                    auto add = [&](uint32_t id) {   // the kMax smallest list indices (lights_sum_in_list_order)
                        if (sorted_insert(ids, id) != 0xffffffffu) dropped = true;
                    };
                    // the big list's candidates, tested once per walk (bigc below)
                    if (!big_over) {
                        for (uint32_t q = 0; q < nbig; ++q)
                            if (bigc[q] >= lo) add(bigc[q]);
                    } else {
                        for (uint32_t q = 0; q < big; ++q) {
                            const uint32_t id = lg_id[q];
                            if (id >= lo && big_hit(g.lg_sph[q])) add(id);
                        }
                    }
                    auto merge_piece = [&](uint32_t gi) {
                        typedef uint32_t u4 __attribute__((ext_vector_type(4)));
                        const u4* sl = reinterpret_cast<const u4*>(slots + (gi - B) * kSlot);
                        RTW_PROBE_LANES(14);
                        const u4 w0 = sl[0], w1 = sl[1];
                        const uint32_t cnt = w0.x;
                        const uint32_t e[7] = {w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
#pragma unroll
                        for (uint32_t q = 0; q < kPieceIds; ++q)
                            if (q < cnt && e[q] >= lo) add(e[q]);
                        if (cnt > kPieceIds) bp = min(bp, e[kPieceIds - 1]);
                    };
                    if (one_pass) {
                        // only the ray's pieces with a candidate (first - B + kp <= 64)
                        uint64_t m = kp ? held >> (first - B) : 0ull;
                        if (kp < 64u) m &= (1ull << kp) - 1ull;
                        for (; m; m &= m - 1ull) merge_piece(first + (uint32_t)__builtin_ctzll(m));
                    } else {
                        for (uint32_t gi = first; gi < first + kp; ++gi) merge_piece(gi);
                    }
                    bound = dropped ? min(bp, ids[kMax - 1]) : bp;
#pragma unroll
                    for (uint32_t q = 0; q < kMax; ++q) n += ids[q] != 0xffffffffu ? 1u : 0u;
                }
                mark(16);
                if constexpr (RTW_COOP_DEAL != 0) {
                    // the owner's summable ids: ids[0..m) (sorted, <= bound)
                    uint32_t m = 0;
                    if (owning) {
#pragma unroll
                        for (uint32_t q = 0; q < kMax; ++q) m += (q < n && ids[q] <= bound) ? 1u : 0u;
                    }
                    uint32_t incl_m = m;
#pragma unroll
                    for (uint32_t off = 1; off < 64; off <<= 1) {
                        const uint32_t v = (uint32_t)__shfl_up((int)incl_m, off);
                        if (lane >= off) incl_m += v;
                    }
                    const uint32_t fm = incl_m - m, T = (uint32_t)__shfl((int)incl_m, 63);
                    for (uint32_t r = 0; r < T; r += 64) {
                        const uint32_t gi = r + lane;
                        uint32_t own = 0;   // the owner of candidate gi: the last lane whose first is <= gi
#pragma unroll
                        for (uint32_t step = 32; step; step >>= 1) {
                            const uint32_t f = (uint32_t)__shfl((int)fm, (int)(own + step));
                            own = f <= gi ? own + step : own;
                        }
                        const uint32_t q = gi - (uint32_t)__shfl((int)fm, (int)own);
                        uint32_t id = 0;
#pragma unroll
                        for (uint32_t k2 = 0; k2 < kMax; ++k2) {
                            const uint32_t v = (uint32_t)bperm_i((int32_t)(k2 < n ? ids[k2] : 0u), (int32_t)own);
                            id = k2 == q ? v : id;
                        }
                        RTW_PROBE_LANES(15);
                        const R val = gi < T ? pdf_at(id, own) : (R)0;
                        // each owner adds its values of this pass, in list order
                        const uint32_t g0 = max(fm, r), g1 = min(fm + m, r + 64u);   // its candidates in this pass
                        const uint32_t q0 = g0 - r, cnt = g1 > g0 ? g1 - g0 : 0u;
                        uint32_t cmax = cnt;
#pragma unroll
                        for (int off = 32; off > 0; off >>= 1) cmax = max(cmax, (uint32_t)__shfl_xor((int)cmax, off));
                        for (uint32_t jq = 0; jq < cmax; ++jq) {
                            const R v = bperm_any(val, (int32_t)((q0 + jq) & 63u));
                            if (jq < cnt) acc = acc + v;
                        }
                    }
                } else {
                    sum_ids(ids, n, bound, acc);
                }
                mark(15);
                if (owning) {
                    if (bound == 0xffffffffu) {
                        more = false;                       // every candidate summed
                        owning = false;
                    } else {
                        lo = bound + 1u;
                        if (bound == bp) {                  // a piece's dropped candidates are next
                            walk_again = true;
                            owning = false;
                        }
                    }
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            mark(15);
            B = Bn;
            if (B >= total) break;
        }
        more = more && walk_again;
    }
    return acc;
}


// the f64 instance: candidates by the f64 path's f32 pre-pass (light_may_hit),
// the pdfs in f64 from the pending ray in the wave's LDS stash
template <typename Mark>
__device__ __forceinline__ double lights_pdf_grid_coop64(const Grid64& sc, bool pend,
                                                         const uint32_t* __restrict__ ray, uint32_t P,
                                                         uint32_t* __restrict__ slots, uint32_t cap_words,
                                                         uint32_t lane, LightWork& lw, Mark&& mark) {
    auto ray_at = [&](uint32_t q) {
        return __longlong_as_double((long long)((uint64_t)ray[(2 * q) * 64 + lane] |
                                                ((uint64_t)ray[(2 * q + 1) * 64 + lane] << 32)));
    };
    auto ray_o = [&]() { return mk(ray_at(0), ray_at(1), ray_at(2)); };
    auto ray_d = [&]() { return mk(ray_at(3), ray_at(4), ray_at(5)); };
    // the grid as a DevScene<float> (only the fields the walk reads)
    DevScene<float> g;
    g.lg_start = sc.lg_start;
    g.lg_sph = sc.lg_sph32;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        g.lg_lo[a] = sc.lo[a];
        g.lg_hi[a] = sc.hi[a];
        g.lg_cell[a] = sc.cell[a];
        g.lg_inv[a] = sc.inv[a];
        g.lg_n[a] = sc.n[a];
    }
    V3<float> of, df;           // the f32 ray
    {
        const LightPre pre(ray_o(), ray_d());
        of = mk(pre.ox, pre.oy, pre.oz);
        df = mk(pre.dx, pre.dy, pre.dz);
    }
    const float ia = __builtin_amdgcn_rcpf(__builtin_fmaf(df.x, df.x, __builtin_fmaf(df.y, df.y, df.z * df.z)));
    auto cand = [&](const R4<float>& L, V3<float> ro, V3<float> rd, float, float ria, float ron, float rdn) {
        return light_may_hit(L.x, L.y, L.z, L.w, ro.x, ro.y, ro.z, rd.x, rd.y, rd.z, ria, ron, rdn);
    };
    auto big_hit = [&](const R4<float>& L) {
        const float ib = __builtin_amdgcn_rcpf(__builtin_fmaf(df.x, df.x, __builtin_fmaf(df.y, df.y, df.z * df.z)));
        const float on = fabsf(of.x) + fabsf(of.y) + fabsf(of.z), dn = fabsf(df.x) + fabsf(df.y) + fabsf(df.z);
        return light_may_hit(L.x, L.y, L.z, L.w, of.x, of.y, of.z, df.x, df.y, df.z, ib, on, dn);
    };
    auto sum_ids = [&](const uint32_t* ids, uint32_t n, uint32_t bound, double& acc) {
        const V3<double> o = ray_o(), d = ray_d();
        for (uint32_t q = 0; q < n; ++q) {
            if (ids[q] > bound) break;
            const R4<double> L = sc.lights[ids[q]];
            acc = acc + sphere_pdf_value(mk(L.x, L.y, L.z), L.w, o, d);
        }
    };
    auto pdf_at = [&](uint32_t id, uint32_t owner) {   // the owner's f64 ray from its stash column
        auto at = [&](uint32_t q) {
            return __longlong_as_double((long long)((uint64_t)ray[(2 * q) * 64 + owner] |
                                                    ((uint64_t)ray[(2 * q + 1) * 64 + owner] << 32)));
        };
        const R4<double> L = sc.lights[id];
        return sphere_pdf_value(mk(L.x, L.y, L.z), L.w, mk(at(0), at(1), at(2)), mk(at(3), at(4), at(5)));
    };
    return lights_pdf_grid_coop_list<double>(g, sc.lg_rec, sc.lg_id, sc.big, of, df, ia, pend, P, slots, cap_words,
                                             lane, lw, cand, big_hit, sum_ids, pdf_at, mark);
}

// Light list with quads (DevScene::lref set): HittableList::pdf_value over
// the mixed list in list order (hittable_list.rs:408-412), reference
// arithmetic per entry; `li` = the sphere lights (LDS-staged or global).
template <typename R>
__device__ __forceinline__ R lights_pdf_mixed(const DevScene<R>& sc, const R4<R>* __restrict__ li, V3<R> o,
                                              V3<R> d) {
    R acc = (R)0;
    for (uint32_t k = 0; k < sc.n_list; ++k) {
        const uint32_t ref = sc.lref[k];
        if (ref & kLrefQuad) {
            acc = acc + quad_pdf_value(sc.lquads + kQuadR * (ref & 0x3fffffffu), o, d);
        } else if (ref & kLrefDefault) {
            acc = acc + (R)0;                      // Hittable::pdf_value default, hittable.rs:175-177
        } else {
            const R4<R> L = li[ref];
            acc = acc + sphere_pdf_value(mk(L.x, L.y, L.z), L.w, o, d);
        }
    }
    return acc;
}

// ---------------------------------------------------------------------------
// Textures (kOptTex kernels): Texture::get_colour, texture.rs:15-102
// ---------------------------------------------------------------------------
__device__ __forceinline__ double fmod_(double a, double b) { return ::fmod(a, b); }
__device__ __forceinline__ float fmod_(float a, float b) { return ::fmodf(a, b); }

// Perlin::noise (perlin.rs:59-82) + perlin_interpolation (:96-108): the
// oracle's rtwo_perlin_noise, term for term (iproduct order, Sum from -0.0)
template <typename R>
__device__ __forceinline__ R perlin_noise(const R4<R>* __restrict__ vec, const uint32_t* __restrict__ perm,
                                          V3<R> p) {
    const R u = p.x - floor_(p.x), v = p.y - floor_(p.y), w = p.z - floor_(p.z);
    const R i = floor_(p.x), j = floor_(p.y), k = floor_(p.z);
    R acc = (R)-0.0;
#pragma unroll
    for (int di = 0; di < 2; ++di) {
        const uint32_t px = perm[perlin_index(i + (R)di)];
#pragma unroll
        for (int dj = 0; dj < 2; ++dj) {
            const uint32_t py = perm[256 + perlin_index(j + (R)dj)];
#pragma unroll
            for (int dk = 0; dk < 2; ++dk) {
                const R4<R> c = vec[px ^ py ^ perm[512 + perlin_index(k + (R)dk)]];
                const R fi = (R)di, fj = (R)dj, fk = (R)dk;
                const V3<R> wv = mk(u - fi, v - fj, w - fk);
                const R term = (fi * u + ((R)1 - fi) * ((R)1 - u)) * (fj * v + ((R)1 - fj) * ((R)1 - v)) *
                               (fk * w + ((R)1 - fk) * ((R)1 - w)) * dot(mk(c.x, c.y, c.z), wv);
                acc = acc + term;
            }
        }
    }
    return acc;
}

// CheckerTexture (nested textures followed iteratively), NoiseTexture
// (0.5 (1 + sin(scale z + 10 turb(p, 7)))), SolidColour
template <typename R>
__device__ V3<R> tex_colour(const DevScene<R>& sc, uint32_t tid, R u, R v, V3<R> p) {
    for (int depth = 0; depth < 64; ++depth) {
        const uint32_t kind = sc.tex_type[tid];
        const R4<R> tp = sc.tex_p[tid];
        if (kind == 1u) {
            const R s = floor_(u * tp.w) + floor_(v * tp.w);
            tid = fmod_(s, (R)2) == (R)0 ? sc.tex_refs[2 * tid] : sc.tex_refs[2 * tid + 1];
            continue;
        }
        if (kind == 2u) {
            const uint32_t q = sc.tex_refs[2 * tid];
            const R4<R>* vec = sc.perlin_vec + 256 * q;
            const uint32_t* perm = sc.perlin_perm + 768 * q;
            R accum = (R)0, weight = (R)1;        // Perlin::turb, perlin.rs:84-94
            V3<R> t = p;
            for (int o = 0; o < 7; ++o) {
                accum = accum + weight * perlin_noise(vec, perm, t);
                t = t * (R)2;
                weight = weight * (R)0.5;
            }
            const R x = rt_sin(tp.w * p.z + accum * (R)10) + (R)1;
            return mk((R)0.5 * x, (R)0.5 * x, (R)0.5 * x);
        }
        return mk(tp.x, tp.y, tp.z);
    }
    return mk((R)NAN, (R)NAN, (R)NAN);
}


// kOpt: compile-time options, chosen per launch by the host
//   kOptRobust   (f32) closest-approach sphere and light tests (far geometry)
//   kOptLightBvh (BVH kernels) light pdf through the light BVH (long light lists)
//   kOptTex      textured materials (DevScene::mat_tex): hit UVs + Texture::get_colour
//   kOptPrims    quads, transformed cuboids and mixed light lists (DevScene::lref); without
//                it the kernel is spheres + planes only (the Book-1 scenes) and carries none
//                of that code -- fewer live registers across the segment loop
//   kOptHit64    (f32 kernels of sphere + plane scenes) f64 ray origin, own-sphere re-hit test,
//                hit t and hit point (sphere_t_ref64): the reference's self-intersection odds
enum : int { kOptRobust = 1, kOptLightBvh = 2, kOptTex = 4, kOptPrims = 8, kOptHit64 = 16 };
// the kernels with wide workgroups (rtw_kernels.h block_waves): f64, tree in
// LDS, spheres + planes, linear light list
template <typename R, int kWorld, int kOpt>
constexpr bool kernel_wide() {
    return sizeof(R) == 8 && kWorld == kWorldBvhLds && (kOpt & (kOptLightBvh | kOptPrims | kOptTex)) == 0;
}
template <typename R, int kWorld, int kOpt>
constexpr uint32_t kernel_waves() { return block_waves(kernel_wide<R, kWorld, kOpt>()); }
// subtree stealing in the f32 while-while kernels (bvh_traverse_steal); 0
// builds them without it (timing comparisons, tools/variants.sh)
// render_kernel: issue priorities in rotation (see the trip loop)
#ifndef RTW_PRIO_ROTATE
#define RTW_PRIO_ROTATE 1
#endif
#ifndef RTW_PRIO_SHIFT
#define RTW_PRIO_SHIFT 12
#endif
#ifndef RTW_STEAL
#define RTW_STEAL 1
#endif
#ifndef RTW_STEAL_TOP
#define RTW_STEAL_TOP 0
#endif
// ray_colour_tail_call's accumulator `res` (camera.rs:459-522): res += mult *
// emitted at every scatter, added to the sample's colour where it ends.
// Kernels for scenes without a DiffuseLight (kEmit false; the host routes a
// scene with one to the kOptPrims kernels) know emitted() = (0, 0, 0) on every
// hit (material.rs:42-44): res starts at +0 and gains mult * (+0), which is
// +0 or -0 -- no change, +0 + -0 = +0 -- while mult is finite and NaN once it
// is not, and then stays NaN.  So res is +0 or NaN per component: three bits
// instead of three registers, and value() is exactly res.
template <typename R, bool kEmit>
struct ResAcc;
template <typename R>
struct ResAcc<R, true> {
    V3<R> v;
    __device__ __forceinline__ void reset() { v = mk<R>(0, 0, 0); }
    __device__ __forceinline__ void add(V3<R> mult, V3<R> emitted) { v = v + mult * emitted; }
    __device__ __forceinline__ V3<R> value() const { return v; }
};
template <typename R>
struct ResAcc<R, false> {
    uint32_t nan;
    __device__ __forceinline__ void reset() { nan = 0; }
    __device__ __forceinline__ void add(V3<R> mult, V3<R>) {   // emitted is (0, 0, 0) here
        nan |= (__builtin_isfinite(mult.x) ? 0u : 1u) | (__builtin_isfinite(mult.y) ? 0u : 2u) |
               (__builtin_isfinite(mult.z) ? 0u : 4u);
    }
    __device__ __forceinline__ V3<R> value() const {
        return mk<R>((nan & 1u) ? (R)NAN : (R)0, (nan & 2u) ? (R)NAN : (R)0, (nan & 4u) ? (R)NAN : (R)0);
    }
};

template <typename R, int kWorld, int kOpt>
// f32: ask for 5 waves per SIMD (<= 96 VGPRs), 4 for the hit64 kernels.
#ifndef RTW_WAVES
#define RTW_WAVES 5
#endif
#ifndef RTW_WAVES_H64
#define RTW_WAVES_H64 4
#endif
// f64 sphere + plane kernels (no quads / cuboids / textures): 4 waves per SIMD
// (128 VGPRs, ~50 spilled: C2 184 -> 174 ms vs 153 VGPRs at 3 waves); the
// other f64 kernels keep the compiler's choice.
#ifndef RTW_WAVES_F64
#define RTW_WAVES_F64 4
#endif
// f64 kernels with the light grid / BVH (C3, C5): 3 waves per SIMD -- the
// cooperative grid walk on top of the f64 path state needs ~170 VGPRs (at 128
// the compiler spilled the loop-carried state at every trip)
#ifndef RTW_WAVES_F64_LBVH
#define RTW_WAVES_F64_LBVH 3
#endif
// f32 (hit64) kernels with the light grid / BVH: 4 waves per SIMD (3, 168
// VGPRs: C3 / C5 f32 +15 % time; profiles/r05_f32_list_waves_ab.jsonl)
#ifndef RTW_WAVES_H64_LBVH
#define RTW_WAVES_H64_LBVH 4
#endif
__global__ void __launch_bounds__((64 * kernel_waves<R, kWorld, kOpt>()), sizeof(R) == 4 ? ((kOpt & kOptHit64) ? ((kOpt & kOptLightBvh) ? RTW_WAVES_H64_LBVH
                                                                                                      : RTW_WAVES_H64)
                                                                             : RTW_WAVES)
                                                         : ((kOpt & (kOptPrims | kOptTex)) ? 1
                                                            : ((kOpt & kOptLightBvh) ? RTW_WAVES_F64_LBVH
                                                                                     : RTW_WAVES_F64)))
    render_kernel(const KParams<R> p) {
    using PR = P<R>;
    constexpr uint32_t kWB = kernel_waves<R, kWorld, kOpt>();   // waves per workgroup
    constexpr uint32_t kBlk = 64 * kWB;
    constexpr bool kRobust = (kOpt & kOptRobust) != 0;
    constexpr bool kLightBvh = (kOpt & kOptLightBvh) != 0 && kWorld >= kWorldBvh;
    constexpr bool kTex = (kOpt & kOptTex) != 0;
    constexpr bool kPrims = (kOpt & kOptPrims) != 0;
    constexpr bool kHit64 = (kOpt & kOptHit64) != 0 && sizeof(R) == 4 && !kTex && !kPrims;
    // DiffuseLight materials only in the kOptPrims / kOptTex kernels (the host
    // routes scenes with one there): the others know emitted() is black
    constexpr bool kEmit = kPrims || kTex;
    extern __shared__ __attribute__((aligned(32))) unsigned char smem[];
    R4<R>* s_sph = reinterpret_cast<R4<R>*>(smem);
    R4<R>* s_li = s_sph + p.sc.n_sph;
    if constexpr (kWorld == kWorldLds) {
        // Stage the sphere list {c, r^2} and the light list into LDS once per
        // workgroup: every lane of every wave then reads sphere k at the same
        // LDS address (a broadcast read) during its closest-hit sweep.
        for (uint32_t k = threadIdx.x; k < p.sc.n_sph; k += kBlk) s_sph[k] = p.sc.sph[k];
        for (uint32_t k = threadIdx.x; k < p.sc.n_lights; k += kBlk) s_li[k] = p.sc.lights[k];
        __syncthreads();
    }
    const R4<R>* __restrict__ sph = kWorld == kWorldLds ? s_sph : p.sc.sph;
    const R4<R>* __restrict__ li = kWorld == kWorldLds ? s_li : p.sc.lights;
    R4<R>* l_li = nullptr;   // kWorldBvhLds: the light list in LDS
    R4<R>* l_lp = nullptr;   // kWorldBvhLds, f32: the light list as pairs in LDS
    R4<float>* l_li32 = nullptr;   // kWorldBvhLds, f64: the lights rounded to f32 (light pre-pass)
    R4<R>* l_bsph64 = nullptr;     // kWorldBvhLds, f64, wide workgroups: the f64 leaf spheres
    R4<R>* l_sph64 = nullptr;      // ... and the f64 spheres in id order (RTW_WIDE_SPH64)
    // World view of the closest-hit query.  kWorldBvhLds: the BVH nodes and
    // the leaf-ordered spheres + ids are copied into LDS once per workgroup
    // (after the traversal stacks), so traversal fetches go to the LDS
    // instead of the vector-memory (TA/L1) path the shading loads use.
    DevScene<R> scw = p.sc;
    if constexpr (kWorld == kWorldBvhLds) {
        unsigned char* base = smem + traversal_lds<R>(p.stack, kLightBvh, kWB);
        // the f32 tree (bvh32) in both precisions: the while-while traversal culls on it
        BvhNode<float>* l_nodes = reinterpret_cast<BvhNode<float>*>(base);
        // the leaf spheres {c, r^2} in f32 (f64: the pre-pass copy bsph32; the
        // f64 candidates are read from the global leaf array)
        R4<float>* l_bsph = reinterpret_cast<R4<float>*>(l_nodes + p.sc.n_nodes);
        uint32_t* l_bid = reinterpret_cast<uint32_t*>(l_bsph + p.sc.n_sph);
        static_assert(sizeof(BvhNode<float>) % 16 == 0, "nodes are copied in 16-B units");
        const uint4* g_nodes = reinterpret_cast<const uint4*>(cull_nodes(p.sc));
        constexpr uint32_t kNode16 = sizeof(BvhNode<float>) / 16;
        for (uint32_t k = threadIdx.x; k < p.sc.n_nodes * kNode16; k += kBlk)
            reinterpret_cast<uint4*>(l_nodes)[k] = g_nodes[k];
        const R4<float>* g_bsph32;
        if constexpr (sizeof(R) == 4) g_bsph32 = p.sc.bsph;
        else g_bsph32 = p.sc.bsph32;
        for (uint32_t k = threadIdx.x; k < p.sc.n_sph; k += kBlk) {
            l_bsph[k] = g_bsph32[k];
            l_bid[k] = p.sc.bid[k];
        }
        // the light list follows, aligned to its element (read by the light pdf / sampling)
        // (offsets from smem, not integer casts of pointers: a pointer rebuilt from an
        // integer loses its LDS address space, and every access through it became a
        // flat instruction -- which waits on the vector-memory counter as well)
        auto lds_after = [&](const void* end, size_t align) {
            const size_t off = (size_t)(reinterpret_cast<const unsigned char*>(end) - smem);
            return smem + ((off + align - 1) & ~(align - 1));
        };
        l_li = reinterpret_cast<R4<R>*>(lds_after(l_bid + ((p.sc.n_sph + 7u) & ~7u), sizeof(R4<R>)));
        for (uint32_t k = threadIdx.x; k < p.sc.n_lights; k += kBlk) l_li[k] = p.sc.lights[k];
        if constexpr (sizeof(R) == 4) {
            // and again as pairs for the packed light test (lights_pdf_sum_pk)
            l_lp = l_li + p.sc.n_lights;
            const uint32_t n = p.sc.n_lights;
            for (uint32_t q = threadIdx.x; 2 * q < n; q += kBlk) {
                const R4<R> A = p.sc.lights[2 * q];
                const bool odd = 2 * q + 1 < n;
                const R4<R> B = odd ? p.sc.lights[2 * q + 1] : R4<R>{0, 0, 0, 0};
                l_lp[2 * q] = R4<R>{A.x, B.x, A.y, B.y};
                l_lp[2 * q + 1] = R4<R>{A.z, B.z, A.w * A.w, odd ? B.w * B.w : (R)-INFINITY};
            }
        } else {
            // the lights rounded to f32 with |radius| (the f32 pre-pass of lights_pdf_sum;
            // a packed-FP32 pre-pass over light pairs measured 1.4 ms slower: r04)
            l_li32 = reinterpret_cast<R4<float>*>(l_li + p.sc.n_lights);
            for (uint32_t k = threadIdx.x; k < p.sc.n_lights; k += kBlk) {
                const R4<R> L = p.sc.lights[k];
                l_li32[k] = R4<float>{(float)L.x, (float)L.y, (float)L.z, fabsf((float)L.w)};
            }
            if constexpr (kernel_wide<R, kWorld, kOpt>()) {
                // wide workgroups: the f64 leaf spheres too, 32-B aligned (the leaf
                // loop's candidates, test_leaf: an LDS read instead of L1 / L2)
                l_bsph64 = reinterpret_cast<R4<R>*>(lds_after(l_li32 + p.sc.n_lights, 32));
                for (uint32_t k = threadIdx.x; k < p.sc.n_sph; k += kBlk) l_bsph64[k] = p.sc.bsph[k];
#if RTW_WIDE_SPH64
                // and in id order (the own-sphere test at the traversal's start)
                l_sph64 = l_bsph64 + p.sc.n_sph;
                for (uint32_t k = threadIdx.x; k < p.sc.n_sph; k += kBlk) l_sph64[k] = p.sc.sph[k];
#endif
            }
        }
        __syncthreads();
        if constexpr (sizeof(R) == 4) {
            scw.bvh = l_nodes;
            scw.bsph = l_bsph;
        } else {
            scw.bvh32 = l_nodes;
            scw.bsph32 = l_bsph;
            if constexpr (kernel_wide<R, kWorld, kOpt>()) {
                scw.bsph = l_bsph64;
                if (RTW_WIDE_SPH64) scw.sph = l_sph64;
            }
        }
        scw.bid = l_bid;
    }
    if constexpr (kWorld == kWorldBvhLds) li = l_li;

    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    // subtree stealing (while-while kernels): this wave's result slots and
    // rendezvous bytes, after the workgroup's traversal stacks
    // only for trees held in LDS: on large trees (C3, C5 from L2 / MALL) the
    // subtrees idle lanes take early are mostly culled later by the owner's
    // closest hit (C5: 9.6 -> 18.4 node visits per segment), and the steady
    // state loses more than the lanes gain (C3 852 -> 875 ms, C5 1536 -> 1751)
    constexpr bool kSteal = RTW_STEAL && kWorld == kWorldBvhLds;
    unsigned char* const steal_area =
        smem + (size_t)kWB * p.stack * 64 * sizeof(int32_t) + wave * kStealLdsPerWave<R>;
    // the light BVH / grid kernels: the wave's light-work counters (u64 light
    // tests, grid cells), right after the traversal area
    unsigned long long* const wcnt =
        reinterpret_cast<unsigned long long*>(smem + traversal_lds<R>(p.stack, false, kWB) + wave * kLightWorkBytes);
    if constexpr (kLightBvh) {
        if (lane < 2) wcnt[lane] = 0ull;
    }
    // the wave's current task (wave-uniform): local tile lt = global 8x8 tile
    // T = lt * nranks + rank at (tx, ty) -- the ranks take the image's tiles
    // round-robin (rtw_tiles_for_rank) -- and chunks [c_begin, c_begin +
    // glen): a pool of 64 glen (pixel, chunk) items
    uint32_t lt = 0, tx = 0, ty = 0, c_begin = 0, glen = 0;
    uint32_t glen_m = 0;          // glen > 1: ceil(2^32 / glen), q / glen = umulhi(q, glen_m) for q < 64 glen
                                  // (2^32 does not fit: glen == 1 is special-cased)
    // The camera, the background and the task parameters are read where they
    // are used (once per sample, miss or task), from the kernarg segment
    // through an opaque pointer: held in SGPRs across the loop they overflow
    // the SGPR file, and the compiler parks them in VGPR lanes and reads them
    // back with v_readlane -- a VALU instruction each, every segment.
    typedef const KParams<R> __attribute__((address_space(4))) KArgs;
    auto kargs = []() {
        const KArgs* k = (const KArgs*)__builtin_amdgcn_kernarg_segment_ptr();
        asm volatile("" : "+s"(k));   // not loop-invariant for the compiler: loaded at each use
        return k;
    };
    // The scene record for a callee, read from the kernel arguments at the call
    // (the fields it uses, by scalar loads) instead of from `p`, whose fields the
    // compiler hoists into SGPRs held across the whole loop -- the light pdf's
    // walks overflow the SGPR file into VGPR lanes and scratch.  (The host pass
    // only type-checks the kernel body: there it is a reference to `p.sc`.)
#if defined(__HIP_DEVICE_COMPILE__)
#define RTW_KARG_SCENE(name) const DevScene<R> name = kargs()->sc
#else
#define RTW_KARG_SCENE(name) const DevScene<R>& name = p.sc
#endif

    auto set_task = [&](uint32_t t) {
        const KArgs* k = kargs();
        if (k->task_table) {   // longest tiles first, cut by cost
            lt = k->task_table[2 * t];
            const uint32_t e = k->task_table[2 * t + 1];
            c_begin = e & 0xFFFFFu;
            glen = e >> 20;
        } else {
            lt = t / k->n_groups;
            const uint32_t cg = t - lt * k->n_groups;
            c_begin = cg * k->group;
            glen = min(c_begin + k->group, k->n_chunks) - c_begin;
        }
        const uint32_t T = k->tile_map ? k->tile_map[lt] : lt * k->nranks + k->rank;   // (global_tile)
        ty = T / k->tiles_x;
        tx = T - ty * k->tiles_x;
        glen_m = glen > 1 ? (uint32_t)((0xFFFFFFFFull + glen) / glen) : 0u;
    };
    // p.persist: every wave takes tasks from a global counter until none are
    // left, and its lanes move on to the next task's items while others still
    // finish the last one -- no per-task drain, one workgroup setup (LDS
    // staging) per resident workgroup.  Else one task per wave (static map).
    bool more = p.persist != 0;       // wave-uniform: the counter may hold tasks
    if (!p.persist) {
        const uint32_t task = blockIdx.x * kWB + wave;
        if (task >= p.n_tasks) return;
        set_task(task);
    }
    // item q -> (pixel px, chunk c): pixel-major (p.item_order 0: q = chunk
    // offset * 64 + px -- the 64 lanes start on the tile's 64 pixels) or
    // sample-major (1: q = px * glen + chunk offset -- the lanes start on a
    // few pixels' consecutive samples: coherent primary rays and first hits).
    // Every item is still one (pixel, chunk) folded in order by the reduce
    // kernel, so the image does not depend on it.
    auto decode = [&](uint32_t qq, uint32_t& px_out, uint32_t& c_out) {
        if (p.item_order) {
            px_out = glen > 1 ? __umulhi(qq, glen_m) : qq;   // qq / glen: exact, qq < 64 glen <= 2^18
            c_out = c_begin + (qq - px_out * glen);
        } else {
            px_out = qq & 63u;
            c_out = c_begin + (qq >> 6);
        }
    };

    const V3<R> zero = mk<R>(0, 0, 0);
    const R tmin = PR::kEps;
    const int32_t nplanes = (int32_t)p.sc.n_planes;
    const int32_t nquads = (int32_t)p.sc.n_quads;
    const int32_t bbase = nplanes + nquads;                  // object ids: planes, quads,
    const int32_t sbase = bbase + (int32_t)p.sc.n_boxes;     // boxes, spheres

    // per-lane item state
    uint32_t q = lane;            // item index in the task's pool
    uint32_t next_q = 0;          // wave-uniform: first unassigned item
    // (kept small: it is live across the whole segment loop) the pixel (i, j)
    // as i | j << 16 (W, H < 2^16, checked by the host), the item's chunk-sum
    // slot lt * 64 + px (its local tile lt = slot >> 6), its chunk c and the
    // current sample s; the chunk's samples end at min((c + 1) chunk, spp)
    uint32_t ij = 0, slot = 0, c = 0, s = 0;
    auto pix_now = [&]() { return (uint64_t)(ij >> 16) * p.W + (ij & 0xffffu); };   // pixel index
    (void)pix_now;                // (probe builds)
    Rng g;
    V3<R> o = zero, d = zero, mult = zero;
    ResAcc<R, kEmit> res;
    res.reset();
    uint32_t depth = 0;
    int32_t self_s = -1;          // isolated sphere the current ray starts on (else -1); kHit64:
                                  // the sphere it starts on, isolated or not
    bool self_iso = false;        // kHit64: self_s is isolated
    V3<double> o64 = {0.0, 0.0, 0.0};   // kHit64: the ray origin in f64
    V3<double> d64 = {0.0, 0.0, 0.0};   // kHit64: the ray direction in f64 (a Metal / Dielectric
                                        // scatter's own f64 result, else dither64 of the f32 one)
    // segments and Lambertian bounces are counted per wave (scalar: a ballot's
    // popcount per trip), node visits and sphere tests per lane (the tile costs)
    uint32_t segs = 0, lambs = 0, nvis = 0, ntest = 0;
    // (counting renders with KParams::cost_time) the clock at the last trip's
    // start and its lanes
    uint64_t trip_clk = 0;
    uint32_t trip_lanes = 0;
    bool active = false, need = true;
    // kCoopGrid (f32 kernels with the light grid, KParams::grid_piece > 0): a
    // Lambertian bounce's light pdf is left pending (`pend`) for the wave's
    // cooperative grid walk at the end of the trip (lights_pdf_grid_coop); the
    // bounce's att * scattering pdf and half its cosine pdf wait with it
    constexpr bool kCoopGrid = kLightBvh && !kPrims;
    RTW_PROBE_WAVE_BEGIN();
    RTW_PROBE_CLK_INIT();
    RTW_PROBE_HIT_INIT();

    auto start_sample = [&]() {
        const KArgs* k = kargs();
        // tile costs (KParams::tile_cost): the sample's work is the lane's counters at
        // its end minus at its start -- subtracted here, added at the end (a
        // u32 sum: exact modulo 2^32, no register kept)
        if (k->tile_cost) {
            if (s < k->cost_spp && !k->cost_time) atomicSub(k->tile_cost + (slot >> 6), nvis + ntest);
        }
        // Camera::get_ray, camera.rs:274-293 + ray_colour_call, camera.rs:439-457
        const uint32_t i = ij & 0xffffu, j = ij >> 16;
        g.seed(k->seed, (uint64_t)j * k->W + i, s);
        R ox = PR::u_incl(g.next(), (R)-0.5, k->u_scale);
        R oy = PR::u_incl(g.next(), (R)-0.5, k->u_scale);
        V3<R> ps = (mk(k->p00[0], k->p00[1], k->p00[2]) + mk(k->du[0], k->du[1], k->du[2]) * ((R)i + ox)) +
                   mk(k->dv[0], k->dv[1], k->dv[2]) * ((R)j + oy);
        const V3<R> center = mk(k->center[0], k->center[1], k->center[2]);
        V3<R> origin = center;
        if (k->defocus) {
            V3<R> qd = unit_disk<R>(g);
            origin = (center + mk(k->disk_u[0], k->disk_u[1], k->disk_u[2]) * qd.x) +
                     mk(k->disk_v[0], k->disk_v[1], k->disk_v[2]) * qd.z;
        }
        o = origin;
        d = ps - origin;
        if constexpr (kHit64) {
            o64 = to64(origin);
            d64 = dither64(d);
        }
        mult = mk<R>(1, 1, 1);
        res.reset();
        RTW_PROBE_HIT_RESET();
        depth = k->max_depth;
        self_s = -1;
        self_iso = false;
    };
    // (wave-uniform) the end of the items this wave may hand out: its task's 64 glen
    uint32_t claim_end = p.persist ? 0u : 64u * glen;
    // Give every lane that needs one a valid item: from the current pool, then
    // (p.persist) from the next task's; none once no task is left.
    auto acquire = [&]() {
        const KArgs* k = kargs();
        for (;;) {
            const uint64_t want = __ballot(need);
            if (want == 0) break;
            if (next_q >= claim_end) {
                uint32_t t = 0xffffffffu;
                if (more) {
                    const uint64_t live = __ballot(true);
                    const uint32_t leader = (uint32_t)__builtin_ctzll(live);
                    if (lane == leader) t = (uint32_t)atomicAdd(k->counters + 6, 1ull);
                    t = (uint32_t)__shfl((int)t, (int)leader);
                }
                if (t >= k->n_tasks) {   // every task is taken: these lanes are done
                    RTW_PROBE_WAVE_DRY();
                    more = false;
                    need = false;
                    break;
                }
                set_task(t);
                RTW_PROBE_WAVE_TASK();
                next_q = 0;
                claim_end = 64u * glen;
                continue;
            }
            if (need) {
                const uint32_t below = __builtin_amdgcn_mbcnt_hi(
                    (uint32_t)(want >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)want, 0u));
                q = next_q + below;
                if (q < claim_end) {
                    uint32_t px;
                    decode(q, px, c);
                    const uint32_t i = tx * kTile + (px & 7u), j = ty * kTile + (px >> 3);
                    if (i < k->W && j < k->H) {
                        ij = i | (j << 16);
                        slot = lt * 64u + px;
                        s = c * k->chunk;
                        active = true;
                        need = false;
                        start_sample();
                    }
                }
            }
            next_q += (uint32_t)__popcll(want);
        }
    };
    // the first 64 items of the first task go to lanes 0..63 in order
    acquire();
    RTW_PROBE_CLK(0);
#if RTW_PRIO_ROTATE
    // Issue priority in rotation.  A SIMD's arbiter favours its oldest wave:
    // with persistent waves, whose ages never change, the wave in slot 0 ran
    // at 1.46x and the one in slot 3 at 0.53x the mean rate (lane-segments per
    // us, profiles/r06c_timeline.jsonl), and the launch ended on slot-3 waves
    // finishing a task taken long before (an 8-rank C2 share: 1 ms after the
    // median wave).  Each wave takes priority (clock / 2^RTW_PRIO_SHIFT + its
    // slot) mod 4 at every trip, so at any time the waves of a SIMD hold
    // different priorities and each holds the highest a quarter of the time.
    uint32_t prio_slot;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(prio_slot));
    prio_slot &= 3u;
#endif

    for (;;) {
        const uint64_t live = __ballot(active);
        if (live == 0) break;
        if (kargs()->cost_time) {
            // wave-time tile costs (counting renders): the last trip's clock cycles,
            // shared by its lanes, added for each lane running a counted sample now
            // (a trip lasts about as long as the one before it)
            const KArgs* k = kargs();
            const uint64_t now = clock64();
            if (trip_lanes && active && s < k->cost_spp)
                atomicAdd(k->tile_cost + (slot >> 6), (uint32_t)(now - trip_clk) / trip_lanes);
            trip_clk = now;
            trip_lanes = (uint32_t)__popcll(live);
        }
#if RTW_PRIO_ROTATE
        {
            const uint32_t pr = ((uint32_t)(wall_clock64() >> RTW_PRIO_SHIFT) + prio_slot) & 3u;
            if (pr == 0) __builtin_amdgcn_s_setprio(0);
            else if (pr == 1) __builtin_amdgcn_s_setprio(1);
            else if (pr == 2) __builtin_amdgcn_s_setprio(2);
            else __builtin_amdgcn_s_setprio(3);
        }
#endif
        segs += (uint32_t)__popcll(live);   // every active lane runs one segment of this trip
        RTW_PROBE_WAVE_TRIP();
        bool lamb = false;                  // the lane's segment ended in a Lambertian scatter
        // (kCoopGrid) this trip's pending light pdf and the bounce's weights: set by
        // the Lambertian branch, consumed by the walk at the end of the same trip --
        // declared per trip, so the compiler does not carry them across trips
        bool pend = false;
        V3<R> pend_aw = zero;
        R pend_ch = (R)0;
        RTW_PROBE_CLK(12);
        RTW_PROBE_LANES(3);
        if (active) {
            RTW_PROBE_LANES(4);
            if constexpr (kHit64) {
                // the f32 ray is the f64 one rounded (dither64 stays within half an
                // f32 ulp): o, d are not kept live across segments
                o = from64<R>(o64);
                d = from64<R>(d64);
            }
            // ---- world.hit(&r, EPSILON..=INFINITY): closest over all primitives
            R tb = (R)INFINITY;
            int32_t best = -1;
            double tb64 = 0.0;            // kHit64: the closest hit's t in f64
            RTW_PROBE_PLANES();
            for (int32_t k = 0; k < nplanes; ++k) {
                R t;
                // f32 kernels: the plane record through a constant-address-space
                // pointer -- its address is wave-uniform, so these are scalar loads
                // (SGPR operands, the scalar cache) instead of a vector load per field
                // whose latency started every segment (hit64 86.2 -> 85.7 ms, plain
                // 58.0 -> 57.5, C3 f32 -1 %; profiles/r06pl_ab.jsonl).  The f64 kernels
                // keep vector loads: the f64 record's SGPRs spilled (C2 f64 +0.3 %).
                typedef const R __attribute__((address_space(4))) KR;
                using PlanePtr = typename std::conditional<sizeof(R) == 4, KR*, const R*>::type;
                PlanePtr pl = (PlanePtr)kargs()->sc.planes + kPlaneR * k;
                // plane_t's one-sided test (plane.rs:62-63) first: it fails for every
                // ray that leaves the Book-1 ground downwards, and then the box test
                // (side-effect free, bounded_hit's first half) cannot change the outcome
                if (!(dot(d, mk(pl[3], pl[4], pl[5])) > PR::kEps)) continue;
                const bool box_hit = aabb_hit_plane(pl + 6, pl + 9, o, d, tmin);
                if (box_hit && plane_t(pl, o, d, tmin, t, p.counters + 4) &&
                    (best < 0 || t < tb)) {
                    tb = t;
                    best = k;
                }
            }
            // quads, each behind its own AABB (bounded_hit, hittable.rs:190-196)
            for (int32_t k = 0; kPrims && k < nquads; ++k) {
                R t;
                const R* Q = kargs()->sc.quads + kQuadR * k;
                if (aabb_hit_ref(Q + 16, Q + 19, o, d, tmin) && quad_t_hit(Q, o, d, tmin, (R)INFINITY, t) &&
                    (best < 0 || t < tb)) {
                    tb = t;
                    best = nplanes + k;
                }
            }
            // transformed cuboids, each behind its world AABB
            for (int32_t k = 0; kPrims && k < (int32_t)kargs()->sc.n_boxes; ++k) {
                R t;
                int qd;
                V3<R> o2, d2;
                const R* B = kargs()->sc.boxes + kBoxR * k;
                if (aabb_hit_ref(B + kBoxLo, B + kBoxHi, o, d, tmin) &&
                    box_t_hit(B, o, d, tmin, (R)INFINITY, t, qd, o2, d2) && (best < 0 || t < tb)) {
                    tb = t;
                    best = bbase + k;
                }
            }
            RTW_PROBE_CLK(1);
            if constexpr (kHit64) {
                // the own sphere's re-hit in f64, the others in f32 (it excluded), the
                // winner's t again in f64
                tb64 = best >= 0 ? (double)tb : (double)INFINITY;
                bool skip = false;
                if (self_s >= 0) {
                    RTW_PROBE_LANES(5);
                    ++ntest;
                    double ts;
                    bool self_hit = sphere_t_ref64(kargs()->sc.sph64[self_s], o64, d64, ts) && ts < tb64;
                    RTW_PROBE_ABL_SELF(self_hit, ts);
                    if (self_hit) {
                        tb64 = ts;
                        tb = (float)ts;
                        best = sbase + self_s;
                        skip = self_iso;          // isolated: provably the closest sphere hit
                    }
                }
                if constexpr (kSteal) {
                    // every active lane calls the traversal: the skipped ones steal work
                    RTW_PROBE_LANES(6);
                    const int32_t prev = best, excl = self_s >= 0 ? sbase + self_s : -1;
                    int32_t* stk_wave = reinterpret_cast<int32_t*>(smem) + wave * p.stack * 64;
                    bvh_closest_excl_steal<kRobust>(scw, sbase, o, d, tmin, tb, best, stk_wave, lane, steal_area,
                                                    nvis, ntest, excl, skip);
                    if (!skip && best != prev && best >= sbase) {
                        if (!sphere_t_ref64(kargs()->sc.sph64[best - sbase], o64, d64, tb64)) tb64 = (double)tb;
                        RTW_PROBE_ABL_WINNER();
                    }
                } else if (!skip) {   // (kernels without stealing)
                    RTW_PROBE_LANES(6);
                    const int32_t prev = best, excl = self_s >= 0 ? sbase + self_s : -1;
                    if constexpr (kWorld >= kWorldBvh) {
                        int32_t* stk = reinterpret_cast<int32_t*>(smem) + wave * p.stack * 64 + lane;
                        constexpr int kKind = kWorld == kWorldBvhLds ? kWorldBvhWW : kWorld;
                        bvh_closest_excl<kKind, kRobust>(scw, sbase, o, d, tmin, tb, best, stk, nvis, ntest, excl);
                    } else {
                        sweep_spheres_excl<kRobust>(sph, kargs()->sc.n_sph, sbase, o, d, tmin, tb, best, excl);
                    }
                    if (best != prev && best >= sbase) {
                        if (!sphere_t_ref64(kargs()->sc.sph64[best - sbase], o64, d64, tb64)) tb64 = (double)tb;
                        RTW_PROBE_ABL_WINNER();
                    }
                }
                // a plane's t in f64 too, so that its hit points lie within f64 rounding
                // of the plane (the one-sided Book-1 ground is never hit from above)
                if (best >= 0 && best < nplanes) tb64 = plane_t_ref64(kargs()->sc.pl64 + 2 * best, o64, d64);
                RTW_PROBE_H64();
            } else if constexpr (kWorld >= kWorldBvh) {
                RTW_PROBE_CLOSEST();
                int32_t* stk = reinterpret_cast<int32_t*>(smem) + wave * p.stack * 64 + lane;
                constexpr int kKind = kWorld == kWorldBvhLds ? kWorldBvhWW : kWorld;
                if constexpr (kSteal) {
                    bvh_closest_steal<kRobust>(scw, sbase, o, d, tmin, tb, best, stk - lane, lane, steal_area,
                                               nvis, ntest, self_s);
                } else {
                    bvh_closest<kKind, kRobust>(scw, sbase, o, d, tmin, tb, best, stk, nvis, ntest, self_s);
                }
            } else {
                sweep_spheres<kRobust>(sph, kargs()->sc.n_sph, sbase, o, d, tmin, tb, best);
            }
            RTW_PROBE_CLK(2);
            RTW_PROBE_SEGMENT();
            RTW_PROBE_HIT(best);

            bool done = false;
            V3<R> col = zero;
            if (best < 0) {
                const KArgs* k = kargs();
                col = mult * mk(k->bg[0], k->bg[1], k->bg[2]) + res.value();   // camera.rs:473-475
                done = true;
            } else {
                // HitRecord::new, hittable.rs:101-129
                V3<R> pnt = o + d * tb;
                V3<double> pnt64 = {0.0, 0.0, 0.0};
                if constexpr (kHit64) {
                    pnt64 = ray_at64(o64, d64, tb64);
                    pnt = mk((float)pnt64.x, (float)pnt64.y, (float)pnt64.z);
                }
                V3<R> outward;
                uint32_t m, mtype;
                R4<R> mp;
                int32_t next_self = -1;
                bool next_iso = false;
                V3<double> n64 = {0.0, 0.0, 0.0};   // kHit64, sphere hits: the f64 outward normal
                bool sph_hit = false;
                bool box_hit = false;
                bool box_front = false;
                R hu = (R)0, hv = (R)0;                            // HitRecord u, v (kTex)
                if (kPrims && best >= bbase && best < sbase) {
                    // Transformed<Cuboid>: the record of the object-space hit,
                    // its point mapped back (transform_point3d); the normal and
                    // front face stay in object space (transformations.rs:14-29)
                    const R* B = kargs()->sc.boxes + kBoxR * (best - bbase);
                    R t2;
                    int qd = 0;
                    V3<R> o2, d2;
                    box_t_hit(B, o, d, tmin, (R)INFINITY, t2, qd, o2, d2);
                    const V3<R> n = q3(B + kQuadR * qd, 12);
                    box_front = dot(d2, n) < (R)0;
                    outward = n;
                    const V3<R> po = o2 + d2 * t2;
                    pnt = mat3_mul(B + kBoxRot, po) + q3(B, kBoxT);
                    m = kargs()->sc.box_mat[best - bbase];
                    mtype = kargs()->sc.mat_type[m];
                    mp = kargs()->sc.mat_p[m];
                    box_hit = true;
                    if constexpr (kTex) {                          // get_quad_uv, object space
                        const R* Q = B + kQuadR * qd;
                        const V3<R> pq = po - q3(Q, 0);
                        hu = dot(cross(pq, q3(Q, 6)), q3(Q, 9));
                        hv = dot(cross(q3(Q, 3), pq), q3(Q, 9));
                    }
                } else if (best < nplanes) {
                    const R* pl = kargs()->sc.planes + kPlaneR * best;
                    outward = mk(pl[3], pl[4], pl[5]);
                    m = kargs()->sc.plane_mat[best];
                    mtype = kargs()->sc.mat_type[m];
                    mp = kargs()->sc.mat_p[m];
                    if constexpr (kTex) plane_uv(pl, pnt, hu, hv);
                } else if (kPrims && best < bbase) {
                    const R* Q = kargs()->sc.quads + kQuadR * (best - nplanes);
                    outward = q3(Q, 12);                           // quadrilateral.rs:97
                    m = kargs()->sc.quad_mat[best - nplanes];
                    mtype = kargs()->sc.mat_type[m];
                    mp = kargs()->sc.mat_p[m];
                    if constexpr (kTex) {                          // get_quad_uv, quadrilateral.rs:58-63
                        const V3<R> pq = pnt - q3(Q, 0);
                        hu = dot(cross(pq, q3(Q, 6)), q3(Q, 9));
                        hv = dot(cross(q3(Q, 3), pq), q3(Q, 9));
                    }
                } else {
                    const uint32_t k = (uint32_t)(best - sbase);
                    const R4<R> sk = kargs()->sc.sph[k];
                    outward = PR::divs(pnt - mk(sk.x, sk.y, sk.z), kargs()->sc.sph_r[k]);  // sphere.rs:82-83
                    // one level of loads: the sphere's material kind and
                    // parameters are copied per sphere (sph_mat word: id,
                    // kind, isolated flag; sph_shade: albedo + fuzz | ior)
                    const uint32_t mw = kargs()->sc.sph_mat[k];
                    m = mw & 0xffffffu;
                    mtype = (mw >> 24) & 0x7fu;
#if RTW_EXP_HITREC_LOAD2
                    {   // (timing experiment) the shading record's load made dependent on sph_mat's
                        uint32_t z;
                        asm volatile("v_and_b32 %0, 0, %1" : "=v"(z) : "v"(mw));
                        mp = kargs()->sc.sph_shade[k + z];
                    }
#else
                    mp = kargs()->sc.sph_shade[k];
#endif
                    next_self = (mw >> 31) ? (int32_t)k : -1;   // bit 31: isolated sphere
                    if constexpr (kHit64) {
                        next_self = (int32_t)k;
                        next_iso = (mw >> 31) != 0;
                        // Metal / Dielectric scatter in f64 from the f64 normal: their
                        // directions decide the next re-hit at the ulp level
                        bool scatter64 = mtype == kMatMetal || mtype == kMatDielectric;
                        RTW_PROBE_ABL_SCATTER(scatter64);
                        if (scatter64) {
                            n64 = sphere_normal64(pnt64, kargs()->sc.sph64[k]);
                            outward = mk((float)n64.x, (float)n64.y, (float)n64.z);
                            sph_hit = true;
                        }
                    }
                    if constexpr (kTex) sphere_uv(outward, hu, hv);
                }
                bool front = box_hit ? box_front : dot(d, outward) < (R)0;
                if constexpr (kHit64) {
                    if (sph_hit) {                                 // the f64 front face and normal
                        front = front64(d64, n64);
                        if (!front) n64 = -n64;
                    }
                }
                const V3<R> nrm = front ? outward : -outward;
                // Material::emitted: DiffuseLight's colour (material.rs:508-514),
                // black for every other material (material.rs:42-44)
                // the material's colour: its texture at (u, v, p) (kTex) or its SolidColour
                V3<R> colour = mk(mp.x, mp.y, mp.z);
                if constexpr (kTex) {
                    if (mtype == kMatDiffuseLight || mtype == kMatLambertian)
                        colour = tex_colour(p.sc, kargs()->sc.mat_tex[m], hu, hv, pnt);
                }
                const V3<R> emitted = kEmit && mtype == kMatDiffuseLight ? colour : zero;
                RTW_PROBE_CLK(3);
                if (kHit64 && sph_hit) {
                    // Metal / Dielectric sphere: the f64 scatter of both in one pass
                    RTW_PROBE_LANES(7);
                    const bool metal = mtype == kMatMetal;
                    bool keep;
                    RTW_PROBE_SCATTER64(specular_dir64(metal, d64, n64, front, kargs()->sc.mat64[m], g2, keep2).y);
                    d64 = specular_dir64<RTW_HIT64_REF_SPHERE != 0>(metal, d64, n64, front, kargs()->sc.mat64[m], g, keep);
                    if (!keep) {
                        col = mult * emitted + res.value();
                        done = true;
                    } else {
                        if (metal) mult = mult * mk(mp.x, mp.y, mp.z);   // Reflect, camera.rs:488-500
                        o = pnt;                          // (Dielectric: mult * (1, 1, 1) = mult)
                        self_s = next_self;
                        self_iso = next_iso;
                        o64 = pnt64;
                        d = from64<R>(d64);
                    }
                    RTW_PROBE_CLK(6);
                } else if (sizeof(R) == 8 && (mtype == kMatMetal || mtype == kMatDielectric)) {
                    // f64: Metal::scatter and Dialectric::scatter (material.rs:407-421,
                    // 458-487) in one pass (specular_dir64 with the reference's
                    // UnitSphere loop and the material's f64 record: 1 / ior and both
                    // faces' Schlick r0 computed on the host with the reference's
                    // operations), so a wave whose lanes hit both runs it once
                    RTW_PROBE_LANES(7);
                    const bool metal = mtype == kMatMetal;
                    bool keep;
                    const V3<double> dir = specular_dir64<true>(metal, to64(d), to64(nrm), front,
                                                                kargs()->sc.mat64[m], g, keep);
                    if (!keep) {
                        col = mult * emitted + res.value();
                        done = true;
                    } else {
                        if (metal) mult = mult * mk(mp.x, mp.y, mp.z);   // Reflect, camera.rs:488-500
                        o = pnt;                                          // (Dielectric: mult * (1, 1, 1) = mult)
                        self_s = next_self;
                        self_iso = next_iso;
                        d = from64<R>(dir);
                    }
                    RTW_PROBE_CLK(6);
                } else if (mtype == kMatMetal) {
                    RTW_PROBE_LANES(7);
                    // Metal::scatter, material.rs:407-421
                    V3<R> refl = reflect(PR::normalize(d), nrm);
                    const V3<R> dir = refl + unit_sphere<R>(g) * mp.w;
                    if (!(dot(dir, nrm) > (R)0)) {
                        col = mult * emitted + res.value();
                        done = true;
                    } else {
                        mult = mult * mk(mp.x, mp.y, mp.z);            // Reflect, camera.rs:488-500
                        o = pnt;
                        self_s = next_self;
                        self_iso = next_iso;
                        if constexpr (kHit64) {
                            o64 = pnt64;
                            d64 = dither64(dir);
                        }
                        d = dir;
                    }
                    RTW_PROBE_CLK(7);
                } else if (mtype == kMatDielectric) {
                    RTW_PROBE_LANES(8);
                    // Dialectric::scatter, material.rs:458-487
                    V3<R> dir;
                    R ratio = front ? PR::div_((R)1, mp.w) : mp.w;
                    V3<R> unit = PR::normalize(d);
                    R cos_t = PR::min_(dot(unit, -nrm), (R)1);
                    R sin_t = PR::sqrt_((R)1 - cos_t * cos_t);
                    bool cannot = ratio * sin_t > (R)1;
                    if (cannot || reflectance(cos_t, ratio) > PR::u_open01(g.next()))
                        dir = reflect(unit, nrm);
                    else
                        dir = refract(unit, nrm, ratio);
                    if constexpr (kHit64) d64 = dither64(dir);
                    // mult * Colour(1, 1, 1) is the identity on every value
                    o = pnt;
                    self_s = next_self;
                    self_iso = next_iso;
                    if constexpr (kHit64) o64 = pnt64;
                    d = dir;
                    RTW_PROBE_CLK(8);
                } else if (mtype == kMatLambertian) {
                    RTW_PROBE_LANES(9);
                    // Lambertian + MixturePdf(HittablePdf(lights), CosinePdf):
                    // material.rs:357-376, pdf.rs:33-101, camera.rs:504-521
                    lamb = true;
                    const V3<R> att = colour;
                    // the normal's Onb (onb.rs:8-35) is built by mixture_direction
                    // for the cosine lanes only; the pdf needs its w = normalize(n)
                    // (computed after the direction: not held across the sampling)
                    V3<R> dir;
                    const bool to_light = PR::u_std(g.next()) < (R)0.5;
                    bool sampled = false;
                    bool nan_dir = false;   // (light kernels) an empty light list: a NaN direction
                    if (to_light && (kargs()->sc.n_list == 0 || (kPrims && kargs()->sc.lref))) {
                        // HittableList::random (hittable_list.rs:414-419): a
                        // uniform light (one gen_index draw), then its random()
                        // (no lref list without kPrims: the light kernels drop that code
                        // and take an empty list's NaN direction below, as a select after
                        // the cosine lobe's draws -- a direction assigned on two paths was
                        // spilled at every Lambertian bounce; the Book-1 kernels keep this
                        // code -- dropped there, the f64 kernel's registers were allocated
                        // worse: +0.5 %)
                        if constexpr (kLightBvh && !kPrims) {
                            nan_dir = true;
                            atomicAdd(p.counters + 5, 1ull);
                        } else if (kargs()->sc.n_list == 0) {
                            // an empty list panics there (:417): counted; the
                            // sample goes on along a NaN direction and ends NaN
                            // at its next world query, as in the oracle
                            sampled = true;
                            atomicAdd(p.counters + 5, 1ull);
                            dir = mk((R)NAN, (R)NAN, (R)NAN);
                        } else {
                            sampled = true;
                            const uint32_t ref = kargs()->sc.lref[g.index(kargs()->sc.n_list)];
                            if (ref & kLrefQuad) {
                                dir = quad_random(kargs()->sc.lquads + kQuadR * (ref & 0x3fffffffu), pnt, g);
                            } else if (ref & kLrefDefault) {
                                dir = mk<R>(1, 0, 0);              // Hittable::random default
                            } else {
                                const R4<R> L = li[ref];
                                dir = sphere_random(mk(L.x, L.y, L.z), L.w, pnt, g);
                            }
                        }
                    }
                    int32_t lsel = -1;   // the sampled light (f32: always counted in the pdf)
                    V3<double> dir64l = {0.0, 0.0, 0.0};   // RTW_HIT64_LAMB64: the f64 direction
                    bool have64 = false;
                    if (!sampled) {
                        // a sphere light (one gen_index draw, then Sphere::random)
                        // or the cosine lobe, in one pass (mixture_direction)
                        R4<R> L = R4<R>{0, 0, 0, 0};
                        const bool tl = to_light && !nan_dir;
                        if (tl) {
                            lsel = (int32_t)g.index(kargs()->sc.n_lights);
                            L = li[lsel];
                        }
                        if constexpr (kHit64 && RTW_HIT64_LAMB64 != 0) {
                            // experiment: the Lambertian direction in f64 from the f64
                            // normal (same words, the f64 kernels' arithmetic)
                            V3<double> nl = to64(nrm);
                            if (best >= sbase) {
                                nl = sphere_normal64(pnt64, kargs()->sc.sph64[best - sbase]);
                                if (!front64(d64, nl)) nl = -nl;
                            }
                            dir64l = mixture_direction<double, RTW_HIT64_TRIG32 != 0>(
                                tl, nl, V3<double>{(double)L.x, (double)L.y, (double)L.z}, (double)L.w, pnt64, g);
                            dir = from64<R>(dir64l);
                            have64 = true;
                        } else {
                            dir = mixture_direction(tl, nrm, mk(L.x, L.y, L.z), L.w, pnt, g);
                        }
                    }
                    if constexpr (kLightBvh && !kPrims) {
                        dir = nan_dir ? mk((R)NAN, (R)NAN, (R)NAN) : dir;
                        dir64l = nan_dir ? V3<double>{(double)NAN, (double)NAN, (double)NAN} : dir64l;
                    }
                    RTW_PROBE_LAMBERT_DIR();
                    RTW_PROBE_CLK(4);
                    const V3<R> ndir = PR::normalize(dir);
                    const V3<R> wn = PR::normalize(nrm);
                    const R cos_w = PR::over_pi(dot(ndir, wn));
                    R acc;                                                // hittable_list.rs:408-412
                    // the light walks of the light BVH / grid kernels: deferred to the end
                    // of the trip (the grid's by the whole wave, the others per lane)
                    if constexpr (kCoopGrid) {
                        const R spdf = PR::max_(PR::over_pi(dot(nrm, ndir)), (R)0);
                        pend = true;
                        pend_aw = att * spdf;
                        pend_ch = PR::max_(cos_w, (R)0) * (R)0.5;
                        res.add(mult, emitted);
                        o = pnt;
                        self_s = next_self;
                        self_iso = next_iso;
                        if constexpr (kHit64) {
                            o64 = pnt64;
                            d64 = have64 ? dir64l : dither64(dir);
                        }
                        d = dir;
                    } else {
                    if (kPrims && kargs()->sc.lref)
                        acc = lights_pdf_mixed(p.sc, li, pnt, dir);
                    else if constexpr (kLightBvh) {
                        LightWork lw;
                        RTW_KARG_SCENE(wsc);
                        acc = kargs()->light_bvh == 2
                                  ? lights_pdf_grid<kRobust>(wsc, pnt, dir, lw)
                                  : lights_pdf_bvh<kRobust>(wsc, pnt, dir,
                                                            reinterpret_cast<int32_t*>(smem) + wave * p.stack * 64 + lane,
                                                            lw);
                        light_work_lane(wcnt, lw);
                    } else if constexpr (kWorld == kWorldBvhLds && sizeof(R) == 4)
                        acc = lights_pdf_sum_pk<kRobust>(li, l_lp, kargs()->sc.n_lights, pnt, dir, lsel);
                    else if constexpr (kWorld == kWorldBvhLds && sizeof(R) == 8)
                        acc = lights_pdf_sum<kRobust>(li, kargs()->sc.n_lights, pnt, dir, l_li32);
                    else
                        acc = lights_pdf_sum<kRobust>(li, kargs()->sc.n_lights, pnt, dir);
                    RTW_PROBE_LIGHT_PDF();
                    RTW_PROBE_CLK(5);
                    // / len; a BVH leaf list multiplies by len and divides again (bvh.rs:67-76, 191-194)
                    R lpdf = PR::div_(acc, (R)p.sc.n_list);
                    if (p.sc.light_flags & 1u) lpdf = PR::div_(lpdf * (R)p.sc.n_list, (R)p.sc.n_list);
                    const R pdf = lpdf * (R)0.5 + PR::max_(cos_w, (R)0) * (R)0.5;
                    const R spdf = PR::max_(PR::over_pi(dot(nrm, ndir)), (R)0);
                    const V3<R> w = PR::divs(att * spdf, pdf);
                    const V3<R> new_mult = mult * w;
                    RTW_PROBE_NAN_LAMBERT(__builtin_isnan(mult.x + mult.y + mult.z),
                                          __builtin_isnan(new_mult.x + new_mult.y + new_mult.z), best);
                    res.add(mult, emitted);
                    mult = new_mult;
                    o = pnt;
                    self_s = next_self;
                    self_iso = next_iso;
                    if constexpr (kHit64) {
                        o64 = pnt64;
                        d64 = have64 ? dir64l : dither64(dir);
                    }
                    d = dir;
                    }
                    RTW_PROBE_CLK(4);
                } else {
                    // Invisible (material.rs:321-325): scatter() == None
                    col = mult * emitted + res.value();
                    done = true;
                }
                if (!done) {
                    depth -= 1;
                    if (depth == 0) {                                  // camera.rs:470-472
                        col = zero + res.value();
                        done = true;
                        if constexpr (kCoopGrid) pend = false;         // its pdf is not needed
                    }
                }
            }
            if (done) {
                // the item's running sum lives in its chunk-sum slot, not in
                // registers: (0 + s_first) on the first sample, then slot + s
                // -- the fold of camera.rs:323-335 in the same order
                const KArgs* k = kargs();
                R* dst = k->partial + ((size_t)slot * k->n_chunks + c) * 3;
                V3<R> prev = zero;
                if (k->chunk > 1) {   // (wave-uniform: one sample per item never reads the slot)
                    if (s != c * k->chunk) prev = mk(dst[0], dst[1], dst[2]);
                }
                const V3<R> part = prev + col;
                dst[0] = part.x;
                dst[1] = part.y;
                dst[2] = part.z;
                if (k->tile_cost) {   // tile costs for the task order: this sample's work
                    if (s < k->cost_spp && !k->cost_time)
                        atomicAdd(k->tile_cost + (slot >> 6), nvis + ntest + kCostPerSegment * (k->max_depth - depth + 1u));
                }
                ++s;
                if (s < min((c + 1u) * k->chunk, k->spp)) {
                    RTW_PROBE_SEED();
                    start_sample();
                RTW_PROBE_LANES(10);
                } else {
                    active = false;
                    need = true;
                }
            }
        }
        RTW_PROBE_CLK(9);
        lambs += (uint32_t)__popcll(__ballot(lamb));
        if constexpr (kCoopGrid) {
            // the deferred Lambertian light pdfs of this trip, by the whole wave;
            // then the path throughput as in the Lambertian branch
            // (wave-uniform) the grid's walk by the whole wave; else -- the light
            // BVH, or the grid with grid_piece 0 -- each lane walks for its own
            // ray here, where less of the path state is live than at the bounce
            const bool coop_walk = kargs()->light_bvh == 2 && kargs()->grid_piece != 0;
            if (!coop_walk && __any(pend)) {
                const V3<R> po = kHit64 ? from64<R>(o64) : o, pd = kHit64 ? from64<R>(d64) : d;
                R acc = (R)0;
                if (pend) {
                    LightWork lw;
                    RTW_KARG_SCENE(wsc);
                    acc = kargs()->light_bvh == 2
                              ? lights_pdf_grid<kRobust>(wsc, po, pd, lw)
                              : lights_pdf_bvh<kRobust>(wsc, po, pd,
                                                        reinterpret_cast<int32_t*>(smem) + wave * p.stack * 64 + lane, lw);
                    light_work_lane(wcnt, lw);
                    R lpdf = PR::div_(acc, (R)p.sc.n_list);
                    if (p.sc.light_flags & 1u) lpdf = PR::div_(lpdf * (R)p.sc.n_list, (R)p.sc.n_list);
                    const R pdf = lpdf * (R)0.5 + pend_ch;
                    mult = mult * PR::divs(pend_aw, pdf);
                    pend = false;
                }
            }
            if (coop_walk && __any(pend)) {
                // The walk's registers come on top of the whole path state: the RNG
                // state and (hit64) the f64 ray wait in the wave's LDS stack area
                // ([word][lane]; the host sizes p.stack >= kCoopStash + 1) instead of
                // being spilled to scratch by the compiler; the pieces' slots follow.
                // (f64: the RNG state and the pending ray (o, d) itself)
                // (f64, RTW_STASH64_EXTRA: also the throughput and the pending
                // bounce's weights -- without them the compiler spilled ~28
                // dwords per lane around every walk)
                constexpr uint32_t kStash = sizeof(R) == 8 ? kCoopStash64 : (kHit64 ? 20u : 8u);
                static_assert(kStash < (sizeof(R) == 8 ? kCoopStash64 : kCoopStash) + 1,
                              "the host's stack minimum covers the stash");
                uint32_t* area = reinterpret_cast<uint32_t*>(smem) + wave * p.stack * 64;
                // hit64: the pending ray is (o64, d64) rounded (o = pnt, d = dir), so o and d
                // need not stay live to here
                const V3<R> po = kHit64 ? from64<R>(o64) : o, pd = kHit64 ? from64<R>(d64) : d;
                auto put = [&](uint32_t k, uint64_t v) {
                    area[(2 * k) * 64 + lane] = (uint32_t)v;
                    area[(2 * k + 1) * 64 + lane] = (uint32_t)(v >> 32);
                };
                auto get = [&](uint32_t k) {
                    return (uint64_t)area[(2 * k) * 64 + lane] | ((uint64_t)area[(2 * k + 1) * 64 + lane] << 32);
                };
                auto dbits = [](double x) { return (uint64_t)__double_as_longlong(x); };
                auto bitsd = [](uint64_t x) { return __longlong_as_double((long long)x); };
                put(0, g.s0);
                put(1, g.s1);
                put(2, g.s2);
                put(3, g.s3);
                if constexpr (kHit64) {
                    put(4, dbits(o64.x)); put(5, dbits(o64.y)); put(6, dbits(o64.z));
                    put(7, dbits(d64.x)); put(8, dbits(d64.y)); put(9, dbits(d64.z));
                } else if constexpr (sizeof(R) == 8) {
                    put(4, dbits(o.x)); put(5, dbits(o.y)); put(6, dbits(o.z));
                    put(7, dbits(d.x)); put(8, dbits(d.y)); put(9, dbits(d.z));
                    if constexpr (RTW_STASH64_EXTRA != 0) {
                        put(10, dbits(mult.x)); put(11, dbits(mult.y)); put(12, dbits(mult.z));
                        put(13, dbits(pend_aw.x)); put(14, dbits(pend_aw.y)); put(15, dbits(pend_aw.z));
                        put(16, dbits(pend_ch));
                    }
                }
                R acc;
                LightWork lw;
                // the walk's sections for the clock probes (RTW_CLOCK): 13 setup, 14 the
                // pieces' walks, 15 the owners' sums
                auto walk_mark = [&](int id) { (void)id; RTW_PROBE_CLK(id); };
                RTW_PROBE_CLK(11);
                if constexpr (sizeof(R) == 8) {
                    // (the pending ray: stash words 4..9, put above)
                    // the grid's fields read from the kernel arguments here (RTW_KARG_SCENE)
                    RTW_KARG_SCENE(wsc);
                    Grid64 gr;
                    gr.lg_start = wsc.lg_start;
                    gr.lg_rec = wsc.lg_rec;
                    gr.lg_sph32 = wsc.lg_sph32;
                    gr.lg_id = wsc.lg_id;
                    gr.lights = wsc.lights;
#pragma unroll
                    for (int a = 0; a < 3; ++a) {
                        gr.lo[a] = (float)wsc.lg_lo[a];
                        gr.hi[a] = (float)wsc.lg_hi[a];
                        gr.cell[a] = (float)wsc.lg_cell[a];
                        gr.inv[a] = (float)wsc.lg_inv[a];
                        gr.n[a] = wsc.lg_n[a];
                    }
                    gr.big = wsc.lg_big;
                    acc = lights_pdf_grid_coop64(gr, pend, area + 8 * 64, kargs()->grid_piece, area + kStash * 64,
                                                 (kargs()->stack - kStash) * 64, lane, lw, walk_mark);
                } else {
                    float* slots = reinterpret_cast<float*>(area + kStash * 64);
                    RTW_KARG_SCENE(wsc);
                    acc = lights_pdf_grid_coop<kRobust>(wsc, pend, po, pd, kargs()->grid_piece, slots,
                                                        (kargs()->stack - kStash) * 64, lane, lw, walk_mark);
                }
                light_work_wave(wcnt, lw, lane);
                g.s0 = get(0);
                g.s1 = get(1);
                g.s2 = get(2);
                g.s3 = get(3);
                if constexpr (kHit64) {
                    o64 = V3<double>{bitsd(get(4)), bitsd(get(5)), bitsd(get(6))};
                    d64 = V3<double>{bitsd(get(7)), bitsd(get(8)), bitsd(get(9))};
                } else if constexpr (sizeof(R) == 8) {
                    o = V3<R>{(R)bitsd(get(4)), (R)bitsd(get(5)), (R)bitsd(get(6))};
                    d = V3<R>{(R)bitsd(get(7)), (R)bitsd(get(8)), (R)bitsd(get(9))};
                    if constexpr (RTW_STASH64_EXTRA != 0) {
                        mult = V3<R>{(R)bitsd(get(10)), (R)bitsd(get(11)), (R)bitsd(get(12))};
                        pend_aw = V3<R>{(R)bitsd(get(13)), (R)bitsd(get(14)), (R)bitsd(get(15))};
                        pend_ch = (R)bitsd(get(16));
                    }
                }
                if (pend) {
                    R lpdf = PR::div_(acc, (R)p.sc.n_list);
                    if (p.sc.light_flags & 1u) lpdf = PR::div_(lpdf * (R)p.sc.n_list, (R)p.sc.n_list);
                    const R pdf = lpdf * (R)0.5 + pend_ch;
                    mult = mult * PR::divs(pend_aw, pdf);
                    pend = false;
                }
            }
            RTW_PROBE_CLK(11);
        }
        acquire();
        RTW_PROBE_CLK(0);
    }
    RTW_PROBE_CLK(10);
    RTW_PROBE_CLK_END();
    RTW_PROBE_WAVE_END();
    // wave-reduce the per-lane counters (segs, lambs are per wave), one atomic per wave
    for (int off = 32; off > 0; off >>= 1) {
        nvis += __shfl_xor(nvis, off);
        ntest += __shfl_xor(ntest, off);
    }
    if (lane == 0 && p.counters) {
        atomicAdd(p.counters + 0, (unsigned long long)segs);
        atomicAdd(p.counters + 1, (unsigned long long)lambs);
        if (nvis) atomicAdd(p.counters + 2, (unsigned long long)nvis);
        if (ntest) atomicAdd(p.counters + 3, (unsigned long long)ntest);
        if constexpr (kLightBvh) {
            if (wcnt[0]) atomicAdd(p.counters + 7, wcnt[0]);
            if (wcnt[1]) atomicAdd(p.counters + 8, wcnt[1]);
        }
    }
}

// Fold the chunk sums of every pixel in chunk order and write the rank's
// packed tiles: out[(lt * 64 + px) * 3], px = ly * 8 + lx (pixels outside the
// image: 0).  The fold accumulates in double whatever R is: with many chunks
// (C4: 4096 spp) an f32 running sum would lose low bits; in f64 mode this is
// the reference's sequential f64 fold (camera.rs:323-335).
// chunks staged per pass: 12 KiB of LDS per wave in f32; f64 12 chunks (19
// KiB: the step 0.24 ms shorter than at 8, profiles/r04_h_fold_window_ab.txt;
// 16 took 25 KiB: six waves per CU, too few to keep the loads in flight)
#ifndef RTW_FOLD_WIN64
#define RTW_FOLD_WIN64 12
#endif
template <typename R>
constexpr uint32_t kFoldWindow = sizeof(R) == 4 ? 16 : RTW_FOLD_WIN64;

template <typename R>
__global__ void __launch_bounds__(64) reduce_chunks_kernel(const KParams<R> p, R* __restrict__ out) {
    constexpr uint32_t kFoldWin = kFoldWindow<R>;
    constexpr uint32_t kFoldRow = kFoldWin * 3 + 1;    // LDS row (odd: no bank conflicts)
    // one wave per tile; a pixel's chunk sums are contiguous (the sample-major
    // item pool hands the lanes consecutive chunks of one pixel, whose sums
    // then fill whole cache lines together), so the wave stages a window of
    // kFoldWin chunks x 64 pixels through LDS with row-contiguous loads and
    // each lane folds its pixel's row in chunk order
    __shared__ R win[64 * kFoldRow];
    const uint32_t lt = blockIdx.x, lane = threadIdx.x;
    const uint32_t T = global_tile(p, lt);
    const uint32_t ty = T / p.tiles_x, tx = T - ty * p.tiles_x;
    const uint32_t i = tx * kTile + (lane & 7), j = ty * kTile + (lane >> 3);
    const size_t row_len = (size_t)p.n_chunks * 3;
    const R* tile = p.partial + (size_t)lt * 64 * row_len;
    double sx = 0, sy = 0, sz = 0;
    constexpr uint32_t kNv = kFoldWin * 3;
    for (uint32_t c0 = 0; c0 < p.n_chunks; c0 += kFoldWin) {
        const uint32_t kw = min(kFoldWin, p.n_chunks - c0), nv = kw * 3;
        const R* src = tile + (size_t)c0 * 3;
        if (kw == kFoldWin) {
            // full window: every lane's kNv loads issued back to back
            R v[kNv];
#pragma unroll
            for (uint32_t it = 0; it < kNv; ++it) {
                const uint32_t idx = it * 64 + lane, r = idx / kNv, col = idx - r * kNv;
                v[it] = src[r * row_len + col];
            }
#pragma unroll
            for (uint32_t it = 0; it < kNv; ++it) {
                const uint32_t idx = it * 64 + lane, r = idx / kNv, col = idx - r * kNv;
                win[r * kFoldRow + col] = v[it];
            }
        } else {
            for (uint32_t idx = lane; idx < 64 * nv; idx += 64) {
                const uint32_t r = idx / nv, col = idx - r * nv;
                win[r * kFoldRow + col] = src[r * row_len + col];
            }
        }
        __syncthreads();
        const R* row = win + lane * kFoldRow;
        for (uint32_t k = 0; k < kw; ++k) {
            sx = sx + (double)row[3 * k];
            sy = sy + (double)row[3 * k + 1];
            sz = sz + (double)row[3 * k + 2];
        }
        __syncthreads();
    }
    if (i >= p.W || j >= p.H) sx = sy = sz = 0;   // never written
    R* dst = out + ((size_t)lt * 64 + lane) * 3;
    dst[0] = (R)sx;
    dst[1] = (R)sy;
    dst[2] = (R)sz;
}

// Un-interleave the ranks' packed tiles into the image [H][W][3]: one thread
// per pixel slot of every global tile T (v = slot[T], or T for the round
// robin: rank v % nranks, its local tile v / nranks).  ranks = nranks
// buffers, rank_stride elements apart.
template <typename R>
__global__ void __launch_bounds__(256) assemble_tiles_kernel(const R* __restrict__ ranks, size_t rank_stride,
                                                             uint32_t nranks, uint32_t W, uint32_t H,
                                                             uint32_t tiles_x, uint32_t n_tiles,
                                                             const uint32_t* __restrict__ slot,
                                                             R* __restrict__ img) {
    const uint32_t gid = blockIdx.x * 256 + threadIdx.x;
    const uint32_t T = gid >> 6, lane = gid & 63;
    if (T >= n_tiles) return;
    const uint32_t ty = T / tiles_x, tx = T - ty * tiles_x;
    const uint32_t i = tx * kTile + (lane & 7), j = ty * kTile + (lane >> 3);
    if (i >= W || j >= H) return;
    const uint32_t v = slot ? slot[T] : T;
    const uint32_t k = v % nranks, lt = v / nranks;
    const R* src = ranks + k * rank_stride + ((size_t)lt * 64 + lane) * 3;
    R* dst = img + ((size_t)j * W + i) * 3;
    dst[0] = src[0];
    dst[1] = src[1];
    dst[2] = src[2];
}

}  // namespace dev

// dynamic LDS above 64 KiB must be allowed per kernel
template <typename R, int kWorld, int kOpt>
inline void allow_lds(size_t lds_bytes) {
    if (lds_bytes > 65536)
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&dev::render_kernel<R, kWorld, kOpt>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_bytes);
}

// Grid of a persistent launch (KParams::persist == kPersistResident): the
// workgroups that fit on the GPU at once for this kernel and LDS size (its
// occupancy x CUs), no more than the tasks need.  More than that only adds
// workgroups that start late and stretch the tail (C2 8-rank share: 2048
// workgroups 15.3 ms, 1024 = resident at 4 waves/SIMD 14.9 ms); co-residency
// is not required (no grid barrier: tasks come from a counter).
template <typename R, int kWorld, int kOpt>
inline uint32_t resident_blocks(uint32_t blocks, size_t lds_bytes) {
    int per_cu = 0, dev = 0, cus = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(
            &per_cu, reinterpret_cast<const void*>(&dev::render_kernel<R, kWorld, kOpt>),
            64 * dev::kernel_waves<R, kWorld, kOpt>(), lds_bytes) !=
            hipSuccess ||
        hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || per_cu < 1 ||
        cus < 1)
        return std::min<uint32_t>(blocks, 2048u);
    return std::min<uint32_t>(blocks, (uint32_t)(per_cu * cus));
}

constexpr int kVariantRan = 1 << 16;
// Launch the render kernel of `world` with options kOpt; returns the variant
// that ran as kVariantRan | (world << 8) | options (the brute-force worlds drop
// the light BVH, textured scenes map to the while-while BVH).
template <typename R, int kOpt>
inline int launch_world(const KParams<R>& p, int world, size_t lds_bytes, hipStream_t stream) {
    // the grid: one task per wave (p.persist 0), a fixed grid (p.persist), or the
    // resident workgroups (kPersistResident), in workgroups of the kernel's size
    auto grid = [&](uint32_t waves) {
        uint32_t b = (p.n_tasks + waves - 1) / waves;
        if (p.persist && p.persist != kPersistResident) b = b < p.persist ? b : p.persist;
        return b;
    };
    uint32_t blocks = 0;
    const size_t stacks = traversal_lds<R>(p.stack, (kOpt & dev::kOptLightBvh) != 0);
    const bool resident = p.persist == kPersistResident;
    constexpr int kBrute = kOpt & ~dev::kOptLightBvh;   // the light BVH needs the BVH kernels' stack
    // textured scenes are small: their kernels exist for the brute-force and
    // binary while-while worlds only (launch_render_impl maps the others)
    if constexpr ((kOpt & dev::kOptTex) != 0) {
        if (world == kWorldBvh4 || world == kWorldBvh) world = kWorldBvhWW;
    }
    // (the light BVH / grid is only chosen with a BVH world: its brute-force
    // cases are never reached, and instantiating them would put copies of the
    // plain brute-force kernels into the f64 light-grid unit)
    if constexpr ((kOpt & dev::kOptLightBvh) != 0) {
        if (world == kWorldLds || world == kWorldGlobal) return -1;
    }
    switch (world) {
    case kWorldLds:
        if constexpr ((kOpt & dev::kOptLightBvh) == 0) {
            allow_lds<R, kWorldLds, kBrute>(lds_bytes);
            blocks = grid(dev::kernel_waves<R, kWorldLds, kBrute>());
            if (resident) blocks = resident_blocks<R, kWorldLds, kBrute>(blocks, lds_bytes);
            hipLaunchKernelGGL((dev::render_kernel<R, kWorldLds, kBrute>), dim3(blocks),
                               dim3(64 * dev::kernel_waves<R, kWorldLds, kBrute>()), lds_bytes,
                               stream, p);
        }
        return kVariantRan | (kWorldLds << 8) | kBrute;
    case kWorldBvhLds:
        allow_lds<R, kWorldBvhLds, kOpt>(lds_bytes);
        blocks = grid(dev::kernel_waves<R, kWorldBvhLds, kOpt>());
        if (resident) blocks = resident_blocks<R, kWorldBvhLds, kOpt>(blocks, lds_bytes);
        hipLaunchKernelGGL((dev::render_kernel<R, kWorldBvhLds, kOpt>), dim3(blocks),
                           dim3(64 * dev::kernel_waves<R, kWorldBvhLds, kOpt>()), lds_bytes,
                           stream, p);
        return kVariantRan | (kWorldBvhLds << 8) | kOpt;
    case kWorldBvh4:
        if constexpr ((kOpt & dev::kOptTex) == 0) {
            blocks = grid(dev::kernel_waves<R, kWorldBvh4, kOpt>());
            if (resident) blocks = resident_blocks<R, kWorldBvh4, kOpt>(blocks, stacks);
            hipLaunchKernelGGL((dev::render_kernel<R, kWorldBvh4, kOpt>), dim3(blocks),
                               dim3(64 * dev::kernel_waves<R, kWorldBvh4, kOpt>()), stacks, stream, p);
        }
        return kVariantRan | (kWorldBvh4 << 8) | kOpt;
    case kWorldBvhWW:
        blocks = grid(dev::kernel_waves<R, kWorldBvhWW, kOpt>());
        if (resident) blocks = resident_blocks<R, kWorldBvhWW, kOpt>(blocks, stacks);
        hipLaunchKernelGGL((dev::render_kernel<R, kWorldBvhWW, kOpt>), dim3(blocks),
                           dim3(64 * dev::kernel_waves<R, kWorldBvhWW, kOpt>()), stacks,
                           stream, p);
        return kVariantRan | (kWorldBvhWW << 8) | kOpt;
    case kWorldBvh:
        if constexpr ((kOpt & dev::kOptTex) == 0) {
            blocks = grid(dev::kernel_waves<R, kWorldBvh, kOpt>());
            if (resident) blocks = resident_blocks<R, kWorldBvh, kOpt>(blocks, stacks);
            hipLaunchKernelGGL((dev::render_kernel<R, kWorldBvh, kOpt>), dim3(blocks),
                               dim3(64 * dev::kernel_waves<R, kWorldBvh, kOpt>()), stacks, stream, p);
        }
        return kVariantRan | (kWorldBvh << 8) | kOpt;
    default:
        if constexpr ((kOpt & dev::kOptLightBvh) == 0) {
            blocks = grid(dev::kernel_waves<R, kWorldGlobal, kBrute>());
            if (resident) blocks = resident_blocks<R, kWorldGlobal, kBrute>(blocks, 0);
            hipLaunchKernelGGL((dev::render_kernel<R, kWorldGlobal, kBrute>), dim3(blocks),
                               dim3(64 * dev::kernel_waves<R, kWorldGlobal, kBrute>()), 0, stream,
                               p);
        }
        return kVariantRan | (kWorldGlobal << 8) | kBrute;
    }
}

// The f64 kernels with the light BVH / grid are compiled in their own unit
// (render_f64_lgrid.hip) without the shared-divisor quotients (RTW_FASTDIV
// 0: C3 f64 +1.1 % with them, profiles/r06c3fd_ab.log); kOpt includes kOptLightBvh
int launch_render_f64_lgrid(const KParams<double>& p, int world, size_t lds_bytes, hipStream_t stream, int kopt);
// the f64 light-grid unit's body (instantiated there only)
template <typename R>
inline int launch_lgrid_impl(const KParams<R>& p, int world, size_t lds_bytes, hipStream_t stream, int kopt) {
    constexpr int T = dev::kOptTex | dev::kOptPrims, Pr = dev::kOptPrims, L = dev::kOptLightBvh;
    switch (kopt) {
    case T | L: return launch_world<R, T | L>(p, world, lds_bytes, stream);
    case Pr | L: return launch_world<R, Pr | L>(p, world, lds_bytes, stream);
    case L: return launch_world<R, L>(p, world, lds_bytes, stream);
    default: return -1;
    }
}

// Options per launch: the f32 sphere-test form (DevScene::robust; f64 keeps
// the reference arithmetic only) and the light BVH (KParams::light_bvh).
// Returns the variant that ran (launch_world's code; 0: no launch), or -1.
template <typename R>
inline int launch_render_impl(const KParams<R>& p, int world, size_t lds_bytes, R* out,
                              hipStream_t stream, hipEvent_t mid) {
    int ran = 0;
    if (p.n_tasks) {
        const bool robust = sizeof(R) == 4 && p.sc.robust;
        const bool lbvh = p.light_bvh != 0;
        // kOptPrims: always for textured kernels; the Book-1 kernels go
        // without when the scene has no quads, cuboids, mixed list or
        // DiffuseLight (their emission accumulator is three bits, ResAcc)
        const bool prims = p.sc.n_quads || p.sc.n_boxes || p.sc.lref || p.sc.emissive;
        constexpr int T = dev::kOptTex | dev::kOptPrims, Pr = dev::kOptPrims;
        if (p.sc.mat_tex) {
            if constexpr (sizeof(R) == 4) {
                if (robust && lbvh) ran = launch_world<R, T | dev::kOptRobust | dev::kOptLightBvh>(p, world, lds_bytes, stream);
                else if (robust) ran = launch_world<R, T | dev::kOptRobust>(p, world, lds_bytes, stream);
                else if (lbvh) ran = launch_world<R, T | dev::kOptLightBvh>(p, world, lds_bytes, stream);
                else ran = launch_world<R, T>(p, world, lds_bytes, stream);
            } else {
                if (lbvh) ran = launch_render_f64_lgrid(p, world, lds_bytes, stream, T | dev::kOptLightBvh);
                else ran = launch_world<R, T>(p, world, lds_bytes, stream);
            }
        } else if constexpr (sizeof(R) == 4) {
            if (prims) {
                if (robust && lbvh) ran = launch_world<R, Pr | dev::kOptRobust | dev::kOptLightBvh>(p, world, lds_bytes, stream);
                else if (robust) ran = launch_world<R, Pr | dev::kOptRobust>(p, world, lds_bytes, stream);
                else if (lbvh) ran = launch_world<R, Pr | dev::kOptLightBvh>(p, world, lds_bytes, stream);
                else ran = launch_world<R, Pr>(p, world, lds_bytes, stream);
            } else {
                constexpr int H = dev::kOptHit64;
                if (p.hit64) {
                    if (robust && lbvh) ran = launch_world<R, H | dev::kOptRobust | dev::kOptLightBvh>(p, world, lds_bytes, stream);
                    else if (robust) ran = launch_world<R, H | dev::kOptRobust>(p, world, lds_bytes, stream);
                    else if (lbvh) ran = launch_world<R, H | dev::kOptLightBvh>(p, world, lds_bytes, stream);
                    else ran = launch_world<R, H>(p, world, lds_bytes, stream);
                } else {
                    if (robust && lbvh) ran = launch_world<R, dev::kOptRobust | dev::kOptLightBvh>(p, world, lds_bytes, stream);
                    else if (robust) ran = launch_world<R, dev::kOptRobust>(p, world, lds_bytes, stream);
                    else if (lbvh) ran = launch_world<R, dev::kOptLightBvh>(p, world, lds_bytes, stream);
                    else ran = launch_world<R, 0>(p, world, lds_bytes, stream);
                }
            }
        } else {
            // f64: the sphere + plane scenes' kernels go without the quad / cuboid code
            // too (156 instead of 176 VGPRs: 3 waves per SIMD instead of 2)
            (void)robust;
            if (prims) {
                if (lbvh) ran = launch_render_f64_lgrid(p, world, lds_bytes, stream, Pr | dev::kOptLightBvh);
                else ran = launch_world<R, Pr>(p, world, lds_bytes, stream);
            } else {
                if (lbvh) ran = launch_render_f64_lgrid(p, world, lds_bytes, stream, dev::kOptLightBvh);
                else ran = launch_world<R, 0>(p, world, lds_bytes, stream);
            }
        }
        if (hipGetLastError() != hipSuccess) return -1;
    }
    if (mid && hipEventRecord(mid, stream) != hipSuccess) return -1;
    if (p.n_local_tiles) {
        hipLaunchKernelGGL((dev::reduce_chunks_kernel<R>), dim3(p.n_local_tiles), dim3(64), 0, stream, p,
                           out);
        if (hipGetLastError() != hipSuccess) return -1;
    }
    return ran;
}

template <typename R>
inline int launch_assemble_impl(const R* ranks, size_t rank_stride, uint32_t nranks, uint32_t W, uint32_t H,
                                const uint32_t* slot, R* img, hipStream_t stream) {
    const uint32_t tiles_x = (W + kTile - 1) / kTile, n_tiles = tiles_x * ((H + kTile - 1) / kTile);
    const uint32_t blocks = (uint32_t)(((uint64_t)n_tiles * 64 + 255) / 256);
    if (blocks) {
        hipLaunchKernelGGL((dev::assemble_tiles_kernel<R>), dim3(blocks), dim3(256), 0, stream, ranks, rank_stride,
                           nranks, W, H, tiles_x, n_tiles, slot, img);
        if (hipGetLastError() != hipSuccess) return -1;
    }
    return 0;
}

}  // namespace rtw
