// render_kernel.hpp -- the gfx950 render kernels, templated on precision R.
//
// Restates the reference's per-pixel / per-sample loop:
//   render_internal / render_lambda   shared/src/camera.rs:315-388
//   Camera::get_ray                   shared/src/camera.rs:274-293
//   ray_colour_tail_call              shared/src/camera.rs:459-522
// as ONE iterative loop per lane ("path regeneration"): a lane owns a pixel
// of its wave's 8x8 tile and walks that pixel's samples [s_begin, s_end) of
// the work item's chunk; every loop trip traces one segment (one world.hit)
// and, when the path ends, deposits the sample into the lane's running sum
// and immediately starts the next sample.  All 64 lanes therefore share each
// trip's closest-hit sweep, whatever the lengths of their individual paths.
//
// The sample sum of a chunk is folded in sample order exactly like
// `(0..spp).map(..).fold(Colour::default(), +)` (camera.rs:323-335); chunk
// sums are folded in chunk order by reduce_chunks_kernel.
#pragma once

#include "rtw_device.hpp"
#include "rtw_kernels.h"

namespace rtw {
namespace dev {

template <typename R>
__device__ __forceinline__ V3<R> v3of(const R* a) { return mk(a[0], a[1], a[2]); }

// One plane, plane.rs:61-76 (one-sided: only rays moving along +n hit it).
template <typename R>
__device__ __forceinline__ bool plane_t(const R* pl, V3<R> o, V3<R> d, R tmin, R& t) {
    V3<R> n = mk(pl[3], pl[4], pl[5]);
    R denom = dot(d, n);
    if (!(denom > P<R>::kEps)) return false;
    V3<R> op = o - mk(pl[0], pl[1], pl[2]);
    R tt = -P<R>::div_(dot(op, n), denom);
    if (!(tmin <= tt && tt <= (R)INFINITY)) return false;
    t = tt;
    return true;
}

template <typename R, bool kLds>
__global__ void __launch_bounds__(kBlock) render_brute_kernel(const KParams<R> p) {
    using PR = P<R>;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    R4<R>* s_sph = reinterpret_cast<R4<R>*>(smem);
    R4<R>* s_li = s_sph + p.sc.n_sph;
    if constexpr (kLds) {
        // Stage the sphere list {c, r^2} and the light list into LDS once per
        // workgroup: every lane of every wave then reads sphere k with the
        // same LDS address (a broadcast read) in its closest-hit sweep.
        for (uint32_t k = threadIdx.x; k < p.sc.n_sph; k += kBlock) s_sph[k] = p.sc.sph[k];
        for (uint32_t k = threadIdx.x; k < p.sc.n_lights; k += kBlock) s_li[k] = p.sc.lights[k];
        __syncthreads();
    }
    const R4<R>* __restrict__ sph = kLds ? s_sph : p.sc.sph;
    const R4<R>* __restrict__ li = kLds ? s_li : p.sc.lights;

    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint32_t item = blockIdx.x * kWavesPerBlock + wave;
    if (item >= p.n_items) return;
    const uint32_t lt = item / p.n_chunks;
    const uint32_t ch = item - lt * p.n_chunks;
    const uint32_t tr = lt / p.tiles_x;
    const uint32_t tx = lt - tr * p.tiles_x;
    const uint32_t ty = tr * p.nranks + p.rank;
    const uint32_t i = tx * kTile + (lane & 7);
    const uint32_t j = ty * kTile + (lane >> 3);
    const bool valid = i < p.W && j < p.H;
    uint32_t s = ch * p.chunk;
    const uint32_t s_end = min(s + p.chunk, p.spp);
    const uint64_t pix = (uint64_t)j * p.W + i;

    const V3<R> center = v3of(p.center), p00 = v3of(p.p00), du = v3of(p.du), dv = v3of(p.dv);
    const V3<R> bg = v3of(p.bg);
    const V3<R> zero = mk<R>(0, 0, 0);
    const R tmin = PR::kEps;

    V3<R> part = zero;             // fold(Colour::default(), +) of this chunk
    uint32_t segs = 0, lambs = 0;
    Rng g;
    V3<R> o = zero, d = zero, mult = zero, res = zero;
    uint32_t depth = 0;
    bool alive = valid && s < s_end;
    if (alive && p.max_depth == 0) {
        // depth == 0 on entry: every sample is Colour::default() + res = 0
        for (; s < s_end; ++s) part = part + (zero + zero);
        alive = false;
    }

    auto start_sample = [&]() {
        // Camera::get_ray, camera.rs:274-293 + ray_colour_call, camera.rs:439-457
        g.seed(p.seed, pix, s);
        R ox = PR::u_incl(g.next(), (R)-0.5, p.u_scale);
        R oy = PR::u_incl(g.next(), (R)-0.5, p.u_scale);
        V3<R> ps = (p00 + du * ((R)i + ox)) + dv * ((R)j + oy);
        V3<R> origin = center;
        if (p.defocus) {
            V3<R> q = unit_disk<R>(g);
            origin = (center + v3of(p.disk_u) * q.x) + v3of(p.disk_v) * q.z;
        }
        o = origin;
        d = ps - origin;
        mult = mk<R>(1, 1, 1);
        res = zero;
        depth = p.max_depth;
    };
    if (alive) start_sample();

    while (alive) {
        // ---- world.hit(&r, EPSILON..=INFINITY): closest over all primitives
        R tb = (R)INFINITY;
        int32_t best = -1;
        for (uint32_t k = 0; k < p.sc.n_planes; ++k) {
            R t;
            if (plane_t(p.sc.planes + 6 * k, o, d, tmin, t) && (best < 0 || t < tb)) {
                tb = t;
                best = (int32_t)k;
            }
        }
        const int32_t nplanes = (int32_t)p.sc.n_planes;
#pragma unroll 4
        for (uint32_t k = 0; k < p.sc.n_sph; ++k) {
            const R4<R> sk = sph[k];
            R t;
            if (sphere_t(mk(sk.x, sk.y, sk.z), sk.w, o, d, tmin, t) && (best < 0 || t < tb)) {
                tb = t;
                best = nplanes + (int32_t)k;
            }
        }
        ++segs;

        bool done = false;
        V3<R> c = zero;
        if (best < 0) {
            c = mult * bg + res;                                   // camera.rs:473-475
            done = true;
        } else {
            // HitRecord::new, hittable.rs:101-129
            V3<R> pnt = o + d * tb;
            V3<R> outward;
            uint32_t m;
            if (best < nplanes) {
                const R* pl = p.sc.planes + 6 * best;
                outward = mk(pl[3], pl[4], pl[5]);
                m = p.sc.plane_mat[best];
            } else {
                const uint32_t k = (uint32_t)(best - nplanes);
                const R4<R> sk = sph[k];
                outward = PR::divs(pnt - mk(sk.x, sk.y, sk.z), p.sc.sph_r[k]);   // sphere.rs:82-83
                m = p.sc.sph_mat[k];
            }
            const bool front = dot(d, outward) < (R)0;
            const V3<R> nrm = front ? outward : -outward;
            const uint32_t mtype = p.sc.mat_type[m];
            const R4<R> mp = p.sc.mat_p[m];
            const V3<R> emitted = zero;                            // material.rs:42-44
            if (mtype == 1) {
                // Metal::scatter, material.rs:407-421
                V3<R> refl = reflect(PR::normalize(d), nrm);
                V3<R> dir = refl + unit_sphere<R>(g) * mp.w;
                if (!(dot(dir, nrm) > (R)0)) {
                    c = mult * emitted + res;
                    done = true;
                } else {
                    mult = mult * mk(mp.x, mp.y, mp.z);
                    o = pnt;
                    d = dir;
                }
            } else if (mtype == 2) {
                // Dialectric::scatter, material.rs:458-487
                R ratio = front ? PR::div_((R)1, mp.w) : mp.w;
                V3<R> unit = PR::normalize(d);
                R cos_t = PR::min_(dot(unit, -nrm), (R)1);
                R sin_t = PR::sqrt_((R)1 - cos_t * cos_t);
                bool cannot = ratio * sin_t > (R)1;
                V3<R> dir;
                if (cannot || reflectance(cos_t, ratio) > PR::u_open01(g.next()))
                    dir = reflect(unit, nrm);
                else
                    dir = refract(unit, nrm, ratio);
                // mult * Colour(1, 1, 1) is the identity on every value
                o = pnt;
                d = dir;
            } else if (mtype == 0) {
                // Lambertian + MixturePdf(HittablePdf(lights), CosinePdf):
                // material.rs:357-376, pdf.rs:33-101, camera.rs:504-521
                ++lambs;
                const V3<R> att = mk(mp.x, mp.y, mp.z);
                const Onb<R> uvw(nrm);
                V3<R> dir;
                if (PR::u_std(g.next()) < (R)0.5) {
                    // HittableList::random (hittable_list.rs:414-419): choose()
                    const uint32_t nl = p.sc.n_lights;
                    uint32_t pick = 0;
                    (void)g.index(1);
                    if (nl == 2) {
                        if (g.index(2) == 0) pick = 1;
                    } else if (nl >= 3) {
                        uint32_t ix = g.index(nl);
                        pick = ix < nl - 1 ? ix + 1 : 0;
                    }
                    const R4<R> L = li[pick];
                    dir = sphere_random(mk(L.x, L.y, L.z), L.w, pnt, g);
                } else {
                    dir = uvw.transform(cosine_hemisphere<R>(g));
                }
                const V3<R> ndir = PR::normalize(dir);
                const R cos_w = PR::over_pi(dot(ndir, uvw.w));
                R acc = (R)0;                                       // hittable_list.rs:408-412
                for (uint32_t k = 0; k < p.sc.n_lights; ++k) {
                    const R4<R> L = li[k];
                    acc = acc + sphere_pdf_value(mk(L.x, L.y, L.z), L.w, pnt, dir);
                }
                const R lpdf = PR::div_(acc, (R)p.sc.n_lights);
                const R pdf = lpdf * (R)0.5 + PR::max_(cos_w, (R)0) * (R)0.5;
                const R spdf = PR::max_(PR::over_pi(dot(nrm, ndir)), (R)0);
                const V3<R> w = PR::divs(att * spdf, pdf);
                const V3<R> new_mult = mult * w;
                res = res + mult * emitted;
                mult = new_mult;
                o = pnt;
                d = dir;
            } else {
                // Invisible (material.rs:321-325): scatter() == None
                c = mult * emitted + res;
                done = true;
            }
            if (!done) {
                depth -= 1;
                if (depth == 0) {                                    // camera.rs:470-472
                    c = zero + res;
                    done = true;
                }
            }
        }
        if (done) {
            part = part + c;
            ++s;
            if (s < s_end) start_sample();
            else alive = false;
        }
    }

    if (valid) {
        R* dst = p.partial + (((size_t)ch * p.n_local_tiles + lt) * 64 + lane) * 3;
        dst[0] = part.x;
        dst[1] = part.y;
        dst[2] = part.z;
    }
    // wave-reduce the counters, one atomic per wave
    for (int off = 32; off > 0; off >>= 1) {
        segs += __shfl_xor(segs, off);
        lambs += __shfl_xor(lambs, off);
    }
    if (lane == 0 && p.counters) {
        atomicAdd(p.counters + 0, (unsigned long long)segs);
        atomicAdd(p.counters + 1, (unsigned long long)lambs);
    }
}

// Fold the chunk sums of every pixel in chunk order and write the rank's
// packed rows: out[(tr * 8 + ly) * W + i][3].
template <typename R>
__global__ void __launch_bounds__(256) reduce_chunks_kernel(const KParams<R> p, R* __restrict__ out) {
    const uint32_t gid = blockIdx.x * 256 + threadIdx.x;
    const uint32_t lt = gid >> 6, lane = gid & 63;
    if (lt >= p.n_local_tiles) return;
    const uint32_t tr = lt / p.tiles_x, tx = lt - tr * p.tiles_x;
    const uint32_t ty = tr * p.nranks + p.rank;
    const uint32_t i = tx * kTile + (lane & 7), ly = lane >> 3, j = ty * kTile + ly;
    if (i >= p.W || j >= p.H) return;
    R sx = 0, sy = 0, sz = 0;
    const size_t stride = (size_t)p.n_local_tiles * 64 * 3;
    const R* src = p.partial + ((size_t)lt * 64 + lane) * 3;
    for (uint32_t c = 0; c < p.n_chunks; ++c) {
        sx = sx + src[0];
        sy = sy + src[1];
        sz = sz + src[2];
        src += stride;
    }
    R* dst = out + ((size_t)(tr * kTile + ly) * p.W + i) * 3;
    dst[0] = sx;
    dst[1] = sy;
    dst[2] = sz;
}

}  // namespace dev

template <typename R>
inline int launch_render_impl(const KParams<R>& p, int accel, size_t lds_bytes, R* out,
                              hipStream_t stream, hipEvent_t mid) {
    (void)accel;
    const uint32_t blocks = (p.n_items + kWavesPerBlock - 1) / kWavesPerBlock;
    if (blocks) {
        if (lds_bytes) {
            hipLaunchKernelGGL((dev::render_brute_kernel<R, true>), dim3(blocks), dim3(kBlock),
                               lds_bytes, stream, p);
        } else {
            hipLaunchKernelGGL((dev::render_brute_kernel<R, false>), dim3(blocks), dim3(kBlock), 0,
                               stream, p);
        }
        if (hipGetLastError() != hipSuccess) return -1;
    }
    if (mid && hipEventRecord(mid, stream) != hipSuccess) return -1;
    const uint32_t rblocks = (p.n_local_tiles * 64 + 255) / 256;
    if (rblocks) {
        hipLaunchKernelGGL((dev::reduce_chunks_kernel<R>), dim3(rblocks), dim3(256), 0, stream, p,
                           out);
        if (hipGetLastError() != hipSuccess) return -1;
    }
    return 0;
}

}  // namespace rtw
