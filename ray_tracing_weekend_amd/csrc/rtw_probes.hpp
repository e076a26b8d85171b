// rtw_probes.hpp -- experiment-only hooks of the render kernel (never in the
// product build: render_kernel.hpp includes this file only when RTW_EXP,
// RTW_TRACE, RTW_PROF, RTW_TIMELINE or RTW_ABL is defined; otherwise every
// RTW_PROBE_* hook is empty).
//
// RTW_ABL (timing ablations of the kOptHit64 parts): 1 = the
// own-sphere re-hit test in f32, 2 = the winner's t from the f32 traversal,
// 3 = Metal / Dielectric scatter in f32, 4 = f32 directions carried into f64
// without the dither.  Timing only: the images are not the product's.
//
// RTW_EXP (tools/exp_cost.sh): repeat one part of the per-segment work so that
// the time difference prices it.  1 = closest-hit query, 2 = light pdf sum,
// 3 = stream seeding, 4 = Lambertian direction sampling, 5 = plane tests,
// 6 = closest-hit query along another direction, 7 = light pdf sum along the
// same direction; f32 kernels with f64 hit points (kOptHit64): 8 = the
// own-sphere f64 test, 9 = the f32 closest-hit query, 10 = the winner's f64 t,
// 11 = the Metal / Dielectric f64 scatter (each along a permuted direction).
// The repeated work feeds a comparison that never holds, so the compiler
// keeps it.
//
// RTW_PROF (tools/lane_profile.py): at each RTW_PROBE_LANES(id) site, count
// the wave passes and the lanes active in them (1 = BVH inner-node step,
// 2 = parked-leaf tests, 3 = segment loop, 4 = active lanes of a trip, 5 =
// own-sphere f64 test, 6 = closest-hit query, 7 = Metal, 8 = Dielectric,
// 9 = Lambertian, 10 = next sample), read back with rtw_probe_lanes_read.
//
// RTW_CLOCK (tools/clock_profile.py): the wave's shader-clock cycles by part
// of the segment loop -- RTW_PROBE_CLK(id) charges the cycles since the last
// probe to part `id` (a ds_add_u64 by the first active lane into the wave's
// LDS slots; the parts a wave runs one after another under different exec
// masks are charged separately), summed over waves into g_clk at the end.
// 0 item pool + sample start, 1 planes, 2 closest hit, 3 hit record,
// 4 Lambertian (direction + throughput), 5 light pdf, 6 f64 specular,
// 7 Metal, 8 Dielectric, 9 sample end, 10 wave tail (no item left),
// 11 cooperative light-grid walk, 12 loop head.
//
// RTW_NANORIGIN (tools/nan_origins.py): per world object, the samples whose
// throughput turned NaN at a Lambertian bounce off that object (g_nan[1 +
// object id]; g_nan[0]: NaN at any other point of the path, counted at the
// sample's end).
//
// RTW_TRACE (tools/trace_paths.py): record every segment of the first
// kTraceSamples samples of one pixel -- the ray (origin, direction) and the
// closest hit (object id, t) -- into a device array the tool reads back with
// rtw_probe_trace_read_f32 / _f64 (exported by the trace build only).
#pragma once

#define RTW_CAT2(a, b) a##b
#define RTW_CAT(a, b) RTW_CAT2(a, b)

#ifndef RTW_EXP
#define RTW_EXP 0
#endif
#ifndef RTW_ABL
#define RTW_ABL 0
#endif

#if RTW_ABL == 4
#define RTW_PROBE_ABL_DITHER(v) return V3<double>{(v).x, (v).y, (v).z}
#else
#define RTW_PROBE_ABL_DITHER(v)
#endif
#if RTW_ABL == 1
#define RTW_PROBE_ABL_SELF(hit, ts) \
    do { \
        R tf_; \
        const R4<R> s_ = p.sc.sph[self_s]; \
        hit = sphere_t(mk(s_.x, s_.y, s_.z), s_.w, o, d, tmin, tf_) && (double)tf_ < tb64; \
        ts = (double)tf_; \
    } while (0)
#else
#define RTW_PROBE_ABL_SELF(hit, ts)
#endif
#if RTW_ABL == 2
#define RTW_PROBE_ABL_WINNER() (tb64 = (double)tb)
#else
#define RTW_PROBE_ABL_WINNER()
#endif
#if RTW_ABL == 3
#define RTW_PROBE_ABL_SCATTER(f64) (f64 = false)
#else
#define RTW_PROBE_ABL_SCATTER(f64)
#endif

#ifdef RTW_TIMELINE
// tools/share_timeline.py: per wave kTlWords words -- {begin, end} wall-clock
// ticks (100 MHz), task count | last task << 32, XCC id | HW_ID << 32, the
// wave's lane-segments, the tick it took its last task, the tick it found the
// task counter dry and its trips after that -- read back with
// rtw_probe_timeline_read
constexpr uint32_t kTlWaves = 1 << 16, kTlWords = 8;
static __device__ unsigned long long g_tl[kTlWaves * kTlWords];
#define RTW_PROBE_WAVE_BEGIN() \
    uint64_t tl_begin_ = wall_clock64(), tl_last_t_ = tl_begin_, tl_dry_t_ = 0; \
    uint32_t tl_tasks_ = 0, tl_last_ = 0, tl_dry_trips_ = 0
#define RTW_PROBE_WAVE_TASK() (++tl_tasks_, tl_last_ = t, tl_last_t_ = wall_clock64())
#define RTW_PROBE_WAVE_DRY() (tl_dry_t_ = tl_dry_t_ ? tl_dry_t_ : wall_clock64())
#define RTW_PROBE_WAVE_TRIP() (tl_dry_trips_ += tl_dry_t_ ? 1u : 0u)
#define RTW_PROBE_WAVE_END() \
    do { \
        const uint32_t w_ = blockIdx.x * kWB + wave; \
        if (lane == 0 && w_ < kTlWaves) { \
            unsigned xcc_, hw_; \
            asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc_)); \
            asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw_)); \
            unsigned long long* r_ = g_tl + (size_t)kTlWords * w_; \
            r_[0] = tl_begin_; \
            r_[1] = wall_clock64(); \
            r_[2] = tl_tasks_ | ((unsigned long long)tl_last_ << 32); \
            r_[3] = (xcc_ & 0xf) | ((unsigned long long)hw_ << 32); \
            r_[4] = segs; \
            r_[5] = tl_last_t_; \
            r_[6] = tl_dry_t_; \
            r_[7] = tl_dry_trips_; \
        } \
    } while (0)
extern "C" int rtw_probe_timeline_read(unsigned long long* out, size_t n, int reset) {
    n = n < (size_t)kTlWaves * kTlWords ? n : (size_t)kTlWaves * kTlWords;
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_tl), n * sizeof(unsigned long long)) != hipSuccess) return -1;
    if (reset) {
        static unsigned long long zero[kTlWaves * kTlWords];
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_tl), zero, sizeof zero) != hipSuccess) return -1;
    }
    return (int)n;
}
#else
#define RTW_PROBE_WAVE_BEGIN()
#define RTW_PROBE_WAVE_TASK()
#define RTW_PROBE_WAVE_DRY()
#define RTW_PROBE_WAVE_TRIP()
#define RTW_PROBE_WAVE_END()
#endif

#if RTW_EXP == 5
#define RTW_PROBE_PLANES() \
    do { \
        for (int32_t k = 0; k < nplanes; ++k) { \
            R t; \
            const R* pl = p.sc.planes + kPlaneR * k; \
            if (aabb_hit_ref(pl + 6, pl + 9, o, mk(d.y, d.x, d.z), tmin) && \
                plane_t(pl, o, mk(d.y, d.x, d.z), tmin, t, nullptr) && t == (R)-7) \
                ++ntest; \
        } \
    } while (0)
#else
#define RTW_PROBE_PLANES()
#endif

#if RTW_EXP == 1 || RTW_EXP == 6
#define RTW_PROBE_CLOSEST() \
    do { \
        { \
            R tb2 = tb; \
            int32_t best2 = best; \
            const V3<R> d2 = RTW_EXP == 6 ? mk(d.z, d.x, d.y) : d; \
            bvh_closest<kWorld == kWorldBvhLds ? kWorldBvhWW : kWorld, kRobust>(scw, sbase, o, d2, tmin, tb2, best2, \
                                reinterpret_cast<int32_t*>(smem) + wave * p.stack * 64 + lane, nvis, \
                                ntest, self_s); \
            ntest += best2 == -7 ? 1u : 0u; \
        } \
    } while (0)
#else
#define RTW_PROBE_CLOSEST()
#endif

#if RTW_EXP == 4
#define RTW_PROBE_LAMBERT_DIR() \
    do { \
        { \
            Rng g2 = g; \
            V3<R> dir2; \
            if (PR::u_std(g2.next()) < (R)0.5) { \
                const R4<R> L = li[g2.index(p.sc.n_lights)]; \
                dir2 = sphere_random(mk(L.x, L.y, L.z), L.w, pnt, g2); \
            } else { \
                dir2 = Onb<R>(nrm).transform(cosine_hemisphere<R>(g2)); \
            } \
            ntest += dir2.x == (R)-7 ? 1u : 0u; \
        } \
    } while (0)
#else
#define RTW_PROBE_LAMBERT_DIR()
#endif

#if RTW_EXP == 2 || RTW_EXP == 7
#define RTW_PROBE_LIGHT_PDF() \
    do { \
        LightWork lw2; \
        if constexpr (kLightBvh) \
            ntest += (p.light_bvh == 2 \
                         ? lights_pdf_grid<kRobust>(p.sc, pnt, RTW_EXP == 7 ? dir : mk(dir.y, dir.z, dir.x), lw2) \
                         : lights_pdf_bvh<kRobust>(p.sc, pnt, RTW_EXP == 7 ? dir : mk(dir.y, dir.z, dir.x), \
                                                   reinterpret_cast<int32_t*>(smem) + wave * p.stack * 64 + \
                                                       lane, lw2)) == (R)-7 ? 1u : 0u; \
        else \
            ntest += lights_pdf_sum<kRobust>(li, p.sc.n_lights, pnt, mk(dir.y, dir.z, dir.x)) == (R)-7 ? 1u : 0u; \
    } while (0)
#else
#define RTW_PROBE_LIGHT_PDF()
#endif

#if RTW_EXP == 3
#define RTW_PROBE_SEED() \
    do { \
        { \
            Rng g2; \
            g2.seed(p.seed ^ 0x55u, pix_now(), s); \
            ntest += (g2.next() & 0xfffu) == 7u ? 1u : 0u; \
        } \
    } while (0)
#else
#define RTW_PROBE_SEED()
#endif

#if RTW_EXP == 8 || RTW_EXP == 9 || RTW_EXP == 10
#define RTW_PROBE_H64() \
    do { \
        const V3<double> dp_ = {d64.y, d64.z, d64.x}; \
        double t2_ = 0.0; \
        if (RTW_EXP == 8 && self_s >= 0) { \
            if (sphere_t_ref64(p.sc.sph64[self_s], o64, dp_, t2_) && t2_ == -7.0) ++ntest; \
        } \
        if (RTW_EXP == 9) { \
            float tb2_ = (float)INFINITY; \
            int32_t b2_ = -1; \
            if constexpr (kWorld >= kWorldBvh) { \
                int32_t* stk2_ = reinterpret_cast<int32_t*>(smem) + wave * p.stack * 64 + lane; \
                bvh_closest_excl<kWorld == kWorldBvhLds ? kWorldBvhWW : kWorld, kRobust>( \
                    scw, sbase, o, mk(d.y, d.z, d.x), tmin, tb2_, b2_, stk2_, nvis, ntest, -1); \
            } \
            if (b2_ == -7) ++ntest; \
        } \
        if (RTW_EXP == 10 && best >= sbase) { \
            if (sphere_t_ref64(p.sc.sph64[best - sbase], o64, dp_, t2_) && t2_ == -7.0) ++ntest; \
        } \
    } while (0)
#else
#define RTW_PROBE_H64()
#endif

#if RTW_EXP == 11
#define RTW_PROBE_SCATTER64(expr) \
    do { \
        bool keep2; \
        Rng g2 = g; \
        (void)keep2; \
        if ((expr) == -7.0) ++ntest; \
    } while (0)
#else
#define RTW_PROBE_SCATTER64(expr)
#endif

#ifdef RTW_TRACE
// build with -DRTW_TRACE=f32 (render_f32.hip) / -DRTW_TRACE=f64 (render_f64.hip):
// each instantiation unit keeps its own trace array and exports its reader
// (this header is included inside namespace rtw::dev)
constexpr uint32_t kTraceSamples = 64, kTraceSegs = 64, kTraceRec = 8;
static __device__ double g_trace[kTraceSamples * kTraceSegs * kTraceRec];
static __device__ unsigned long long g_trace_pix = ~0ull;
// set the traced pixel (j * W + i) and clear the array / copy it out (n doubles)
extern "C" int RTW_CAT(rtw_probe_trace_set_, RTW_TRACE)(unsigned long long pix) {
    static double zero[kTraceSamples * kTraceSegs * kTraceRec];
    for (auto& z : zero) z = -2.0;
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_trace), zero, sizeof zero) != hipSuccess) return -1;
    return hipMemcpyToSymbol(HIP_SYMBOL(g_trace_pix), &pix, sizeof pix) == hipSuccess ? 0 : -1;
}
extern "C" int RTW_CAT(rtw_probe_trace_read_, RTW_TRACE)(double* out, size_t n) {
    n = n < (size_t)kTraceSamples * kTraceSegs * kTraceRec
            ? n : (size_t)kTraceSamples * kTraceSegs * kTraceRec;
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_trace), n * sizeof(double)) == hipSuccess ? (int)n : -1;
}
// {object id (-1 miss), t, origin xyz, direction xyz} of segment max_depth - depth
#define RTW_PROBE_SEGMENT() \
    do { \
        if (pix_now() == g_trace_pix && s < kTraceSamples && p.max_depth - depth < kTraceSegs) { \
            double* rec = g_trace + ((size_t)s * kTraceSegs + (p.max_depth - depth)) * kTraceRec; \
            double t64 = (double)tb, ox = (double)o.x, oy = (double)o.y, oz = (double)o.z; \
            if constexpr (kHit64) { t64 = tb64; ox = o64.x; oy = o64.y; oz = o64.z; } \
            rec[0] = (double)best; rec[1] = t64; rec[2] = ox; rec[3] = oy; rec[4] = oz; \
            rec[5] = (double)d.x; rec[6] = (double)d.y; rec[7] = (double)d.z; \
        } \
    } while (0)
#else
#define RTW_PROBE_SEGMENT()
#endif

#ifdef RTW_PROF
static __device__ unsigned long long g_lanes[2 * 16];
#define RTW_PROBE_LANES(id) \
    do { \
        const uint64_t m_ = __ballot(true); \
        if ((uint32_t)__lane_id() == (uint32_t)__builtin_ctzll(m_)) { \
            atomicAdd(&g_lanes[2 * (id)], (unsigned long long)__popcll(m_)); \
            atomicAdd(&g_lanes[2 * (id) + 1], 1ull); \
        } \
    } while (0)
extern "C" int RTW_CAT(rtw_probe_lanes_read_, RTW_PROF)(unsigned long long* out, int reset) {
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_lanes), sizeof g_lanes) != hipSuccess) return -1;
    if (reset) {
        static unsigned long long zero[2 * 16];
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_lanes), zero, sizeof zero) != hipSuccess) return -1;
    }
    return 0;
}
#else
#define RTW_PROBE_LANES(id)
#endif

#ifdef RTW_CLOCK
constexpr int kClkParts = 20;
static __device__ unsigned long long g_clk[kClkParts];
#define RTW_PROBE_CLK_INIT() \
    __shared__ unsigned long long clk_lds_[kWB][kClkParts]; \
    if (lane < (uint32_t)kClkParts) clk_lds_[wave][lane] = 0; \
    uint64_t clk_t_ = __builtin_amdgcn_s_memtime()
#define RTW_PROBE_CLK(id) \
    do { \
        const uint64_t n_ = __builtin_amdgcn_s_memtime(); \
        const uint64_t m_ = __ballot(true); \
        if ((uint32_t)__lane_id() == (uint32_t)__builtin_ctzll(m_)) \
            atomicAdd(&clk_lds_[wave][(id)], (unsigned long long)(n_ - clk_t_)); \
        clk_t_ = n_; \
    } while (0)
#define RTW_PROBE_CLK_END() \
    do { \
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront"); \
        __builtin_amdgcn_wave_barrier(); \
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront"); \
        if (lane < (uint32_t)kClkParts) atomicAdd(&g_clk[lane], clk_lds_[wave][lane]); \
    } while (0)
extern "C" int RTW_CAT(rtw_probe_clock_read_, RTW_CLOCK)(unsigned long long* out, int reset) {
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_clk), sizeof g_clk) != hipSuccess) return -1;
    if (reset) {
        static unsigned long long zero[kClkParts];
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_clk), zero, sizeof zero) != hipSuccess) return -1;
    }
    return 0;
}
#else
#define RTW_PROBE_CLK_INIT()
#define RTW_PROBE_CLK(id)
#define RTW_PROBE_CLK_END()
#endif

#ifdef RTW_NANORIGIN
constexpr int kNanSlots = 1 << 16;
static __device__ unsigned long long g_nan[kNanSlots];
#define RTW_PROBE_NAN_LAMBERT(was, now, obj) \
    do { \
        if (!(was) && (now) && (uint32_t)(obj) + 1u < (uint32_t)kNanSlots) atomicAdd(&g_nan[1 + (obj)], 1ull); \
    } while (0)
// and the segments' closest hits per object (slot 1 + id; slot 0: misses),
// and in the second half those that hit the object the previous segment hit
// (a re-hit of the surface the ray starts on: "acne")
static __device__ unsigned long long g_hit[kNanSlots];
#define RTW_PROBE_HIT_INIT() int32_t hit_prev_ = -2
#define RTW_PROBE_HIT_RESET() hit_prev_ = -2
#define RTW_PROBE_HIT(obj) \
    do { \
        if ((uint32_t)((obj) + 1) < (uint32_t)kNanSlots / 2u) { \
            atomicAdd(&g_hit[1 + (obj)], 1ull); \
            if ((obj) >= 0 && (obj) == hit_prev_) atomicAdd(&g_hit[kNanSlots / 2 + 1 + (obj)], 1ull); \
        } \
        hit_prev_ = (obj); \
    } while (0)
extern "C" int RTW_CAT(rtw_probe_hit_read_, RTW_NANORIGIN)(unsigned long long* out, size_t n, int reset) {
    n = n < (size_t)kNanSlots ? n : (size_t)kNanSlots;
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_hit), n * sizeof(unsigned long long)) != hipSuccess) return -1;
    if (reset) {
        static unsigned long long zero[kNanSlots];
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_hit), zero, sizeof zero) != hipSuccess) return -1;
    }
    return (int)n;
}
extern "C" int RTW_CAT(rtw_probe_nan_read_, RTW_NANORIGIN)(unsigned long long* out, size_t n, int reset) {
    n = n < (size_t)kNanSlots ? n : (size_t)kNanSlots;
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_nan), n * sizeof(unsigned long long)) != hipSuccess) return -1;
    if (reset) {
        static unsigned long long zero[kNanSlots];
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_nan), zero, sizeof zero) != hipSuccess) return -1;
    }
    return (int)n;
}
#else
#define RTW_PROBE_NAN_LAMBERT(was, now, obj)
#define RTW_PROBE_HIT(obj)
#define RTW_PROBE_HIT_INIT()
#define RTW_PROBE_HIT_RESET()
#endif
