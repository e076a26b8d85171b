// rtw_device.hpp -- device-side math, RNG and sampling for the gfx950 render
// kernels.  Templated on the arithmetic type R (float = speed mode, double =
// parity mode).  Reference functions restated here are cited as
// path:line relative to N9199/ray_tracing_weekend.
//
// Parity mode (R = double) is compiled with -ffp-contract=off and keeps the
// reference's operation order exactly, so its results can be compared bit
// for bit with the CPU oracle.  Speed mode (R = float) keeps the same
// algorithm and RNG draw order but uses FMA contraction and the native
// v_sqrt/v_rcp/v_rsq/v_sin/v_cos instructions.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rtw {
namespace dev {

template <typename R>
struct V3 {
    R x, y, z;
};

template <typename R>
__device__ __forceinline__ V3<R> mk(R x, R y, R z) { return V3<R>{x, y, z}; }
template <typename R>
__device__ __forceinline__ V3<R> operator+(V3<R> a, V3<R> b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
template <typename R>
__device__ __forceinline__ V3<R> operator-(V3<R> a, V3<R> b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
template <typename R>
__device__ __forceinline__ V3<R> operator-(V3<R> a) { return {-a.x, -a.y, -a.z}; }
template <typename R>
__device__ __forceinline__ V3<R> operator*(V3<R> a, R s) { return {a.x * s, a.y * s, a.z * s}; }
template <typename R>
__device__ __forceinline__ V3<R> operator*(V3<R> a, V3<R> b) { return {a.x * b.x, a.y * b.y, a.z * b.z}; }
// vec.rs:70-72: (x*x' + y*y') + z*z'
template <typename R>
__device__ __forceinline__ R dot(V3<R> a, V3<R> b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
// vec.rs:76-82
template <typename R>
__device__ __forceinline__ V3<R> cross(V3<R> a, V3<R> b) {
    return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}

// ---------------------------------------------------------------------------
// Precision-specific primitives
// ---------------------------------------------------------------------------
template <typename R>
struct P;

// ---------------------------------------------------------------------------
// Exact f64 quotients that share a divisor (Vec3 / scalar, Vec3::normalize)
// ---------------------------------------------------------------------------
// The compiler's IEEE a / b on gfx950 is
//   B = div_scale(b, b, a); y = rcp(B); A, vcc = div_scale(a, b, a);
//   y = fma(y, fma(-B, y, 1), y) twice; q = A y; r = fma(-B, q, A);
//   fixup(div_fmas(r, y, q, vcc), b, a).
// div_scale returns its operand unchanged with vcc = 0 unless a, b or a / b
// is near the ends of the exponent range (or b = 0: then the fixup alone
// decides); with both exponents in [-382, 384] it never rescales, so the
// sequence is fixup(fma(r, y, q), b, a) with y a function of b alone -- the
// SAME instructions on the same values, hence the same bits.  Three
// quotients by one b then pay for one reciprocal instead of three (and no
// div_scale), 17 f64 instructions instead of 33.  Zeros, infinities and NaNs
// pass the range test (frexp_exp gives 0) and are decided by div_fixup from
// a and b alone, as in the full sequence; any lane outside the range takes
// the full division (a wave-uniform skip when none is).  RTW_FASTDIV 0: the
// plain `/` everywhere.
#ifndef RTW_FASTDIV
#define RTW_FASTDIV 1
#endif
__device__ __forceinline__ double recip_nr(double b) {
    double y = __builtin_amdgcn_rcp(b);
    y = __builtin_fma(y, __builtin_fma(-b, y, 1.0), y);
    return __builtin_fma(y, __builtin_fma(-b, y, 1.0), y);
}
__device__ __forceinline__ double div_by(double a, double b, double y) {
    const double q = a * y;
    const double r = __builtin_fma(-b, q, a);
    return __builtin_amdgcn_div_fixup(__builtin_fma(r, y, q), b, a);
}
// frexp exponent + 382, as unsigned: <= 766 iff the exponent is in [-382, 384]
__device__ __forceinline__ uint32_t div_rng(double x) { return (uint32_t)(__builtin_amdgcn_frexp_exp(x) + 382); }
// {x, y, z} / b, each quotient the IEEE one bit for bit
__device__ __forceinline__ V3<double> div3(double x, double y, double z, double b) {
#if RTW_FASTDIV
    const uint32_t m = max(max(div_rng(x), div_rng(y)), max(div_rng(z), div_rng(b)));
    if (__builtin_expect(m <= 766u, 1)) {
        const double yb = recip_nr(b);
        return V3<double>{div_by(x, b, yb), div_by(y, b, yb), div_by(z, b, yb)};
    }
#endif
    return V3<double>{x / b, y / b, z / b};
}

// The sin / cos kernel coefficients (P<double>::k_sin / k_cos) and rt_sin's reduction constants are fdlibm's:
//   Copyright (C) 1993 by Sun Microsystems, Inc. All rights reserved.
//   Developed at SunSoft, a Sun Microsystems, Inc. business.
//   Permission to use, copy, modify, and distribute this software is freely
//   granted, provided that this notice is preserved.
template <>
struct P<double> {
    static constexpr double kPi = 3.14159265358979323846;
    static constexpr double kTau = 2.0 * 3.14159265358979323846;
    static constexpr double kEps = 2.220446049250313080847e-16;  // f64::EPSILON
    static constexpr double kEpsF64 = 2.220446049250313080847e-16;
    __device__ static __forceinline__ double sqrt_(double x) { return __builtin_sqrt(x); }
    __device__ static __forceinline__ double div_(double a, double b) { return a / b; }
    __device__ static __forceinline__ double over_pi(double a) {
#if RTW_FASTDIV >= 2
        // (experiment) the fast quotient with a constant reciprocal of pi: the compiler folds
        // rcp(pi) to RN(1 / pi), so the result is the IEEE one by Markstein's theorem
        // (y = RN(1 / b), q = RN(a y) within an ulp: RN(q + (a - b q) y) = RN(a / b))
        if (__builtin_expect(div_rng(a) <= 766u, 1)) return div_by(a, kPi, recip_nr(kPi));
#endif
        return a / kPi;
    }
    __device__ static __forceinline__ double min_(double a, double b) { return __builtin_fmin(a, b); }
    __device__ static __forceinline__ double max_(double a, double b) { return __builtin_fmax(a, b); }
    // vec.rs:86-94: self / self.length()
    __device__ static __forceinline__ V3<double> normalize(V3<double> a) {
        double l = sqrt_(dot(a, a));
        return div3(a.x, a.y, a.z, l);
    }
    __device__ static __forceinline__ V3<double> divs(V3<double> a, double s) {
        return div3(a.x, a.y, a.z, s);
    }
    // rand 0.8.6 Standard for f64: (v >> 11) * 2^-53
    __device__ static __forceinline__ double u_std(uint64_t v) {
        return (1.0 / 9007199254740992.0) * (double)(v >> 11);
    }
    // 2 * u_std(v) - 1 (UnitSphere's / UnitDisk's coordinate, utils.rs:99-144)
    // without the integer conversion: with b = bit 63 of v and D = 1 + m 2^-52
    // built from bits 11..62 (m), (v >> 11) 2^-52 - 1 = D - (2 - b), and both
    // roundings are exact (Sterbenz), so the two forms agree bit for bit
    // (tests/test_rng_forms.py checks the identity over 2^20 words and the edges)
    __device__ static __forceinline__ double u_pm1(uint64_t v) {
        const uint32_t hi = (uint32_t)(v >> 32), lo = (uint32_t)v;
        const uint32_t dlo = __builtin_amdgcn_alignbit(hi, lo, 11);
        const uint32_t dhi = 0x3FF00000u | ((hi >> 11) & 0xFFFFFu);
        const uint32_t chi = 0x40000000u - ((hi >> 31) << 20);
        return __hiloint2double((int)dhi, (int)dlo) - __hiloint2double((int)chi, 0);
    }
    __device__ static __forceinline__ double unit12(uint64_t v) {
        return __longlong_as_double((long long)((v >> 12) | 0x3FF0000000000000ULL));
    }
    // rand 0.8.6 Open01 for f64
    __device__ static __forceinline__ double u_open01(uint64_t v) {
        return unit12(v) - (1.0 - kEps / 2.0);
    }
    // rand 0.8.6 UniformFloat::sample: value0_1 * scale + low
    __device__ static __forceinline__ double u_incl(uint64_t v, double low, double scale) {
        double v01 = unit12(v) - 1.0;
        return v01 * scale + low;
    }
    // fdlibm __kernel_sin / __kernel_cos after an exact quadrant reduction of r
    // (identical arithmetic to the oracle's rtwo_sincos_2pi)
    __device__ static __forceinline__ double k_sin(double x) {
        const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
                     S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
                     S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
        double z = x * x;
        double v = z * x;
        double r = S2 + z * (S3 + z * (S4 + z * (S5 + z * S6)));
        return x + v * (S1 + z * r);
    }
    __device__ static __forceinline__ double k_cos(double x) {
        const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
                     C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
                     C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
        double z = x * x;
        double r = z * (C1 + z * (C2 + z * (C3 + z * (C4 + z * (C5 + z * C6)))));
        double ax = __builtin_fabs(x);
        if (ax < 0.3) return 1.0 - (0.5 * z - (z * r));
        double qx;
        if (ax > 0.78125) {
            qx = 0.28125;
        } else {
            unsigned long long b = (unsigned long long)__double_as_longlong(ax);
            b = (b - 0x0020000000000000ULL) & 0xFFFFFFFF00000000ULL;
            qx = __longlong_as_double((long long)b);
        }
        double hz = 0.5 * z - qx;
        double a = 1.0 - qx;
        return a - (hz - z * r);
    }
    __device__ static __forceinline__ void sincos_2pi(double r, double* s, double* c) {
        double q = __builtin_rint(r * 4.0);
        double f = r - q * 0.25;
        double x = f * kTau;
        double ks = k_sin(x), kc = k_cos(x);
        switch (((long long)q) & 3) {
            case 0: *s = ks; *c = kc; break;
            case 1: *s = kc; *c = -ks; break;
            case 2: *s = -ks; *c = -kc; break;
            default: *s = -kc; *c = ks; break;
        }
    }
};

template <>
struct P<float> {
    static constexpr float kPi = 3.14159265358979323846f;
    static constexpr float kInvPi = 0.318309886183790671538f;
    static constexpr float kEps = 2.220446049250313080847e-16f;  // same t_min as f64 (2^-52)
    static constexpr float kEpsF64 = 2.220446049250313080847e-16f;
    __device__ static __forceinline__ float sqrt_(float x) { return __builtin_amdgcn_sqrtf(x); }
    __device__ static __forceinline__ float div_(float a, float b) { return a * __builtin_amdgcn_rcpf(b); }
    __device__ static __forceinline__ float over_pi(float a) { return a * kInvPi; }
    __device__ static __forceinline__ float min_(float a, float b) { return __builtin_fminf(a, b); }
    __device__ static __forceinline__ float max_(float a, float b) { return __builtin_fmaxf(a, b); }
    __device__ static __forceinline__ V3<float> normalize(V3<float> a) {
        float k = __builtin_amdgcn_rsqf(dot(a, a));
        return {a.x * k, a.y * k, a.z * k};
    }
    __device__ static __forceinline__ V3<float> divs(V3<float> a, float s) {
        float k = __builtin_amdgcn_rcpf(s);
        return {a.x * k, a.y * k, a.z * k};
    }
    // The f32 draws are the top bits of the SAME 64-bit words the f64 path
    // uses, so both precisions follow the same sample paths until rounding
    // separates them.
    __device__ static __forceinline__ float u_std(uint64_t v) {
        return (float)(uint32_t)(v >> 40) * 5.9604644775390625e-08f;  // 2^-24
    }
    __device__ static __forceinline__ float u_open01(uint64_t v) {
        return (float)(uint32_t)(v >> 41) * 1.1920928955078125e-07f + 5.9604644775390625e-08f;
    }
    __device__ static __forceinline__ float u_incl(uint64_t v, float low, float /*scale*/) {
        return (float)(uint32_t)(v >> 40) * 5.9604644775390625e-08f + low;
    }
    // v_sin_f32 / v_cos_f32 take their argument in revolutions: sin(2*pi*r)
    __device__ static __forceinline__ void sincos_2pi(float r, float* s, float* c) {
        *s = __builtin_amdgcn_sinf(r);
        *c = __builtin_amdgcn_cosf(r);
    }
};

// ---------------------------------------------------------------------------
// RNG: xoshiro256++ (rand 0.8.6 SmallRng) seeded per (pixel, sample) through
// splitmix64 -- identical to the oracle's rtwo_rng_seed / rtwo_rng_next.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
// (x << k) | (x >> (64 - k)) as two v_alignbit_b32 (the compiler's shift / or
// form takes three instructions); k >= 32 rotates the swapped halves by k - 32
template <int k>
__device__ __forceinline__ uint64_t rotl(uint64_t x) {
    static_assert(k > 0 && k < 64 && k != 32, "rotation count");
    const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
    if constexpr (k < 32)
        return ((uint64_t)__builtin_amdgcn_alignbit(hi, lo, 32 - k) << 32) | __builtin_amdgcn_alignbit(lo, hi, 32 - k);
    else
        return ((uint64_t)__builtin_amdgcn_alignbit(lo, hi, 64 - k) << 32) | __builtin_amdgcn_alignbit(hi, lo, 64 - k);
}

// a ^ b ^ c in one gfx950 v_bitop3_b32 (truth table 0x96: odd parity)
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
__device__ __forceinline__ uint64_t xor3(uint64_t a, uint64_t b, uint64_t c) {
    return ((uint64_t)xor3((uint32_t)(a >> 32), (uint32_t)(b >> 32), (uint32_t)(c >> 32)) << 32) |
           xor3((uint32_t)a, (uint32_t)b, (uint32_t)c);
}

struct Rng {
    uint64_t s0, s1, s2, s3;
    __device__ __forceinline__ void seed(uint64_t seed, uint64_t pixel, uint64_t sample) {
        uint64_t k = mix64(seed + 0x9E3779B97F4A7C15ULL * (pixel + 1));
        k = mix64(k ^ (0xD1B54A32D192ED03ULL * (sample + 1)));
        k += 0x9E3779B97F4A7C15ULL; s0 = mix64(k);
        k += 0x9E3779B97F4A7C15ULL; s1 = mix64(k);
        k += 0x9E3779B97F4A7C15ULL; s2 = mix64(k);
        k += 0x9E3779B97F4A7C15ULL; s3 = mix64(k);
    }
    // xoshiro256++ next(): s2 ^= s0; s3 ^= s1; s1 ^= s2; s0 ^= s3; s2 ^= t;
    // s3 = rotl(s3, 45) -- with the chained xors folded into three-input ones
    // (s1' = s1 ^ s2 ^ s0, s0' = s0 ^ s3 ^ s1, s2' = s2 ^ s0 ^ t): the same
    // state, 15 instructions instead of 17
    __device__ __forceinline__ uint64_t next() {
        const uint64_t result = rotl<23>(s0 + s3) + s0;
        const uint64_t t = s1 << 17;
        const uint64_t n1 = xor3(s1, s2, s0), n0 = xor3(s0, s3, s1), n2 = xor3(s2, s0, t);
        s3 = rotl<45>(s3 ^ s1);
        s0 = n0;
        s1 = n1;
        s2 = n2;
        return result;
    }
    // gen_range(0..n) for u32 (rand 0.8.6 sample_single_inclusive), next_u32 = next >> 32
    __device__ __forceinline__ uint32_t index(uint32_t n) {
        uint32_t zone = (n << __builtin_clz(n)) - 1u;
        for (;;) {
            uint32_t v = (uint32_t)(next() >> 32);
            uint64_t m = (uint64_t)v * (uint64_t)n;
            if ((uint32_t)m <= zone) return (uint32_t)(m >> 32);
        }
    }
};

// ---------------------------------------------------------------------------
// Geometry helpers
// ---------------------------------------------------------------------------
template <typename R>
__device__ __forceinline__ V3<R> reflect(V3<R> v, V3<R> n) {   // vec.rs:105-107
    R d = dot(v, n);
    V3<R> n2 = n * (R)2;
    return v - n2 * d;
}
template <typename R>
__device__ __forceinline__ V3<R> refract(V3<R> v, V3<R> n, R eta) {   // vec.rs:111-116
    R cos_theta = P<R>::min_(dot(v, -n), (R)1);
    V3<R> perp = (v + n * cos_theta) * eta;
    V3<R> par = n * (-(P<R>::sqrt_((R)1 - dot(perp, perp))));
    return perp + par;
}

template <typename R>
struct Onb {   // geometry/src/onb.rs:8-35
    V3<R> u, v, w;
    __device__ __forceinline__ explicit Onb(V3<R> n) {
        w = P<R>::normalize(n);
        V3<R> a = __builtin_fabs((double)w.x) > 0.9 ? mk<R>(0, 1, 0) : mk<R>(1, 0, 0);
        v = P<R>::normalize(cross(w, a));
        u = cross(w, v);
    }
    // (0..3).map(|i| e[i] * x[i]).sum() folds from Vec3::default()
    __device__ __forceinline__ V3<R> transform(V3<R> x) const {
        V3<R> acc = mk<R>(0, 0, 0);
        acc = acc + u * x.x;
        acc = acc + v * x.y;
        acc = acc + w * x.z;
        return acc;
    }
};

// utils.rs:99-122 (UnitSphere): a uniform point of the open unit ball.
// f64 (parity mode): the reference's rejection sampling in [-1, 1)^3; the
// shuffle of the three i.i.d. coordinates (utils.rs:116) leaves their law
// unchanged and is not drawn (as in the oracle).
// f32 (speed mode): the same law sampled directly from three uniforms --
// radius u^(1/3), direction by Archimedes (z uniform in [-1, 1], azimuth
// uniform) -- so a wave no longer loops until its last Metal lane has been
// accepted (pi/6 per try: ~4.5 tries for a wave's ~15 Metal lanes, ~500 VALU
// instructions per segment of the wave).  It draws 3 words
// instead of 3 per try: f32 and f64 paths part at a fuzzy-Metal bounce
// (they part within a few bounces anyway).
template <typename R>
__device__ __forceinline__ V3<R> unit_sphere(Rng& g) {
    if constexpr (sizeof(R) == 4) {
        const float z = 2.f * P<float>::u_std(g.next()) - 1.f;
        const float az = P<float>::u_std(g.next());
        const float u = P<float>::u_std(g.next());
        // u^(1/3) as exp2(log2(u) / 3); u = 0 gives r = 0
        const float r = u > 0.f ? __builtin_amdgcn_exp2f(__builtin_amdgcn_logf(u) * (1.f / 3.f)) : 0.f;
        float s, c;
        P<float>::sincos_2pi(az, &s, &c);
        const float rxy = r * __builtin_amdgcn_sqrtf(__builtin_fmaxf(1.f - z * z, 0.f));
        return mk(rxy * c, rxy * s, r * z);
    } else {
        // Each try decides |p|^2 < 1 first from the words' top 32 bits in f32:
        // with hi = v >> 32, a = hi - 2^31 (exact as a signed int) is within
        // 2^6 + 2^31 2^-31 of x 2^31 once rounded to f32, so a^2 + b^2 + c^2
        // (f32 FMAs) is within 8e-7 2^62 of |p|^2 2^62; outside 1 +- 4e-6 the
        // f64 test has the same outcome, inside it (p ~ 3e-6 per try) the
        // f64 test runs.  The accepted try's f64 coordinates are built once.
        constexpr float kLo = (float)((1.0 - 4e-6) * 4611686018427387904.0);   // 2^62
        constexpr float kHi = (float)((1.0 + 4e-6) * 4611686018427387904.0);
        auto top = [](uint64_t v) { return (float)(int32_t)((uint32_t)(v >> 32) ^ 0x80000000u); };
        uint64_t w0, w1, w2;
        for (;;) {
            w0 = g.next();
            w1 = g.next();
            w2 = g.next();
            const float a = top(w0), b = top(w1), c = top(w2);
            const float l = __builtin_fmaf(a, a, __builtin_fmaf(b, b, c * c));
            if (l < kLo) break;
            if (l <= kHi) {
                const V3<R> out = mk(P<R>::u_pm1(w0), P<R>::u_pm1(w1), P<R>::u_pm1(w2));
                if (dot(out, out) < (R)1) break;
            }
        }
        return mk(P<R>::u_pm1(w0), P<R>::u_pm1(w1), P<R>::u_pm1(w2));
    }
}
// utils.rs:124-144
template <typename R>
__device__ __forceinline__ V3<R> unit_disk(Rng& g) {
    if constexpr (sizeof(R) == 8) {
        // the f32 pre-decision of unit_sphere (two coordinates: a^2 + b^2 is
        // within 6e-7 2^62 of |p|^2 2^62)
        constexpr float kLo = (float)((1.0 - 4e-6) * 4611686018427387904.0);
        constexpr float kHi = (float)((1.0 + 4e-6) * 4611686018427387904.0);
        auto top = [](uint64_t v) { return (float)(int32_t)((uint32_t)(v >> 32) ^ 0x80000000u); };
        uint64_t w0, w1;
        for (;;) {
            w0 = g.next();
            w1 = g.next();
            const float a = top(w0), b = top(w1);
            const float l = __builtin_fmaf(a, a, b * b);
            if (l < kLo) break;
            if (l <= kHi) {
                const V3<R> out = mk<R>(P<R>::u_pm1(w0), 0, P<R>::u_pm1(w1));
                if (dot(out, out) < (R)1) break;
            }
        }
        return mk<R>(P<R>::u_pm1(w0), 0, P<R>::u_pm1(w1));
    }
    for (;;) {
        R x, z;
        if constexpr (sizeof(R) == 8) {      // 2 u - 1 from the word's bits (u_pm1, exact)
            x = P<R>::u_pm1(g.next());
            z = P<R>::u_pm1(g.next());
        } else {
            x = (R)2 * P<R>::u_std(g.next()) - (R)1;
            z = (R)2 * P<R>::u_std(g.next()) - (R)1;
        }
        V3<R> out = mk<R>(x, 0, z);
        if (dot(out, out) < (R)1) return out;
    }
}
// utils.rs:146-161
template <typename R>
__device__ __forceinline__ V3<R> cosine_hemisphere(Rng& g) {
    R r1 = P<R>::u_std(g.next());
    R r2 = P<R>::u_std(g.next());
    R s, c;
    P<R>::sincos_2pi(r1, &s, &c);
    R sq = P<R>::sqrt_(r2);
    return mk(c * sq, s * sq, P<R>::sqrt_((R)1 - r2));
}

// Sphere::hit root selection, sphere.rs:61-80.  r2 = radius * radius.
template <typename R>
__device__ __forceinline__ bool sphere_t(V3<R> c, R r2, V3<R> o, V3<R> d, R tmin, R& t) {
    V3<R> oc = o - c;
    R a = dot(d, d);
    R half_b = dot(d, oc);
    R cc = dot(oc, oc) - r2;
    R disc = half_b * half_b - a * cc;
    if (!(disc > (R)0)) return false;
    R sq = P<R>::sqrt_(disc);
    R root = P<R>::div_(-half_b - sq, a);
    if (!(tmin <= root && root <= (R)INFINITY)) {
        root = P<R>::div_(-half_b + sq, a);
        if (!(tmin <= root && root <= (R)INFINITY)) return false;
    }
    t = root;
    return true;
}

// Sphere::pdf_value, sphere.rs:101-111
template <typename R>
__device__ __forceinline__ R sphere_pdf_value(V3<R> c, R radius, V3<R> o, V3<R> d) {
    R t;
    if (!sphere_t(c, radius * radius, o, d, (R)0, t)) return (R)0;
    V3<R> co = c - o;
    R dist2 = dot(co, co);
    if constexpr (sizeof(R) == 4) {
        // f32: 1 - sqrt(1 - x) = x / (1 + sqrt(1 - x)) -- for a far light
        // (x = r^2/d^2 below 2^-24) the reference form rounds to 0 and the
        // pdf to inf in f32
        const float x = radius * radius * __builtin_amdgcn_rcpf(dist2);
        const float one_minus_cos = x * __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_sqrtf(1.f - x));
        return __builtin_amdgcn_rcpf((2.f * P<float>::kPi) * one_minus_cos);
    } else {
        R cos_theta_max = P<R>::sqrt_((R)1 - P<R>::div_(radius * radius, dist2));
        R solid_angle = ((R)2 * P<R>::kPi) * ((R)1 - cos_theta_max);
        return P<R>::div_((R)1, solid_angle);
    }
}

// Sphere::random, sphere.rs:114-127
template <typename R>
__device__ __forceinline__ V3<R> sphere_random(V3<R> c, R radius, V3<R> o, Rng& g) {
    V3<R> direction = c - o;
    R distance = P<R>::sqrt_(dot(direction, direction));
    Onb<R> uvw(direction);
    R r1 = P<R>::u_std(g.next());
    R r2 = P<R>::u_std(g.next());
    R s, cph;
    P<R>::sincos_2pi(r2, &s, &cph);
    if constexpr (sizeof(R) == 4) {
        // f32: w = 1 - z = r1 (1 - cos_max) and 1 - z^2 = w (2 - w), both
        // without cancellation for the narrow cone of a far light
        const float q = radius * radius * __builtin_amdgcn_rcpf(distance * distance);
        const float w = r1 * (q * __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_sqrtf(1.f - q)));
        const float z = 1.f - w;
        const float sxy = __builtin_amdgcn_sqrtf(w * (2.f - w));
        return uvw.transform(mk(cph * sxy, s * sxy, z));
    } else {
        R z = (R)1 + r1 * (P<R>::sqrt_((R)1 - P<R>::div_(radius * radius, distance * distance)) - (R)1);
        R x = cph * P<R>::sqrt_((R)1 - z * z);
        R y = s * P<R>::sqrt_((R)1 - z * z);
        return uvw.transform(mk(x, y, z));
    }
}

// The Lambertian mixture's direction (MixturePdf::generate, pdf.rs:91-96)
// for a light list of spheres: to_light -> Sphere::random of light L
// (sphere.rs:113-127, as sphere_random), else CosinePdf::generate in the
// normal's frame (pdf.rs:45-48, as cosine_hemisphere).  Both draw r1, r2,
// take an azimuth from one and a height from the other and rotate by a
// frame, so one code path serves both: the lanes of a wave that took either
// branch run it together (one pass instead of two).  Per lane the words and
// the operations are those of the separate sampler, so the result is the
// same bit for bit (f64: the oracle's rtwo_sphere_random /
// rtwo_cosine_hemisphere).
// kTrig32 (the f32 kernels' f64 Lambertian direction, RTW_HIT64_LAMB64): the
// azimuth's sine and cosine by the f32 hardware instructions, the rest in R
template <typename R, bool kTrig32 = false>
__device__ __forceinline__ V3<R> mixture_direction(bool to_light, V3<R> n, V3<R> c, R radius, V3<R> o, Rng& g) {
    // one Onb per lane: the light direction's (Sphere::random) or the normal's
    // (CosinePdf::generate), built by the same code for both
    const V3<R> direction = c - o;
    const Onb<R> f(to_light ? direction : n);
    const V3<R> fu = f.u, fv = f.v, fw = f.w;
    R q = (R)0;   // light: r^2 / distance^2
    if (to_light) {
        const R distance = P<R>::sqrt_(dot(direction, direction));
        if constexpr (sizeof(R) == 4) q = radius * radius * __builtin_amdgcn_rcpf(distance * distance);
        else q = P<R>::div_(radius * radius, distance * distance);
    }
    const R r1 = P<R>::u_std(g.next());
    const R r2 = P<R>::u_std(g.next());
    R s, cph;
    if constexpr (kTrig32 && sizeof(R) == 8) {
        float sf, cf;
        P<float>::sincos_2pi((float)(to_light ? r2 : r1), &sf, &cf);
        s = (R)sf;
        cph = (R)cf;
    } else {
        P<R>::sincos_2pi(to_light ? r2 : r1, &s, &cph);
    }
    const R t = P<R>::sqrt_((R)1 - (to_light ? q : r2));   // light: sqrt(1 - r^2/d^2); cosine: z
    R z, sxy;
    if constexpr (sizeof(R) == 4) {
        // light: w = 1 - z = r1 (1 - cos_max), 1 - z^2 = w (2 - w) (see sphere_random)
        const float w = r1 * (q * __builtin_amdgcn_rcpf(1.f + t));
        z = to_light ? 1.f - w : t;
        sxy = __builtin_amdgcn_sqrtf(to_light ? w * (2.f - w) : r2);
    } else {
        z = to_light ? (R)1 + r1 * (t - (R)1) : t;
        sxy = P<R>::sqrt_(to_light ? (R)1 - z * z : r2);
    }
    const V3<R> x = mk(cph * sxy, s * sxy, z);
    V3<R> acc = mk<R>(0, 0, 0);   // Onb::transform's fold
    acc = acc + fu * x.x;
    acc = acc + fv * x.y;
    acc = acc + fw * x.z;
    return acc;
}

// ---------------------------------------------------------------------------
// Quad (quadrilateral.rs), on the staged record Q (rtw_kernels.h kQuadR):
// Q[0..2] q, [3..5] u, [6..8] v, [9..11] w, [12..14] unit normal, [15] area.
// Operation order as the oracle's quad_new / quad_hit_t.
// ---------------------------------------------------------------------------
template <typename R>
__device__ __forceinline__ V3<R> q3(const R* Q, int k) { return mk(Q[k], Q[k + 1], Q[k + 2]); }

// Quad::hit, quadrilateral.rs:79-100: two-sided, t in [tmin, tmax], (alpha,
// beta) = get_quad_uv in [0, 1] inclusive
template <typename R>
__device__ __forceinline__ bool quad_t_hit(const R* Q, V3<R> o, V3<R> d, R tmin, R tmax, R& t) {
    const V3<R> n = q3(Q, 12);
    const R denom = dot(d, n);
    if (!(fabs(denom) > P<R>::kEpsF64)) return false;
    const R tt = -P<R>::div_(dot(o - q3(Q, 0), n), denom);
    if (!(tt >= tmin && tt <= tmax)) return false;
    const V3<R> pq = (o + d * tt) - q3(Q, 0);
    const V3<R> w = q3(Q, 9);
    const R alpha = dot(cross(pq, q3(Q, 6)), w);
    const R beta = dot(cross(q3(Q, 3), pq), w);
    if (!(alpha >= (R)0 && alpha <= (R)1 && beta >= (R)0 && beta <= (R)1)) return false;
    t = tt;
    return true;
}

// Quad::pdf_value, quadrilateral.rs:102-112
template <typename R>
__device__ __forceinline__ R quad_pdf_value(const R* Q, V3<R> o, V3<R> d) {
    R t;
    if (!quad_t_hit(Q, o, d, (R)0, (R)INFINITY, t)) return (R)0;
    const V3<R> n0 = q3(Q, 12);
    const V3<R> n = dot(d, n0) < (R)0 ? n0 : -n0;               // HitRecord::new
    const R distance_squared = t * t * dot(d, d);
    const R cosine = fabs(P<R>::div_(dot(d, n), P<R>::sqrt_(dot(d, d))));
    return P<R>::div_(distance_squared, cosine * Q[15]);
}

// Quad::random, quadrilateral.rs:114-118 (u's Open01 draw first)
template <typename R>
__device__ __forceinline__ V3<R> quad_random(const R* Q, V3<R> o, Rng& g) {
    const R r1 = P<R>::u_open01(g.next());
    const R r2 = P<R>::u_open01(g.next());
    const V3<R> p = (q3(Q, 0) + q3(Q, 3) * r1) + q3(Q, 6) * r2;
    return p - o;
}

// Dialectric::reflectance, material.rs:450-454; powi(5) = x * ((x*x)*(x*x))
template <typename R>
__device__ __forceinline__ R reflectance(R cosine, R ref_idx) {
    R r0 = P<R>::div_((R)1 - ref_idx, (R)1 + ref_idx);
    r0 = r0 * r0;
    R x = (R)1 - cosine;
    R x2 = x * x;
    R p5 = x * (x2 * x2);
    return r0 + ((R)1 - r0) * p5;
}

// ---------------------------------------------------------------------------
// Textures (texture.rs, perlin.rs)
// ---------------------------------------------------------------------------
// f64::sin of a general argument: fdlibm's medium Cody-Waite reduction by
// pi/2 and __kernel_sin/__kernel_cos with the tail -- the oracle's rtwo_sin
// operation for operation (|x| >= 2^19 pi/2 falls back to the library).
__device__ __forceinline__ double k_sin_y(double x, double y) {
    const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
                 S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
                 S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
    double z = x * x;
    double v = z * x;
    double r = S2 + z * (S3 + z * (S4 + z * (S5 + z * S6)));
    return x - ((z * (0.5 * y - v * r) - y) - v * S1);
}
__device__ __forceinline__ double k_cos_y(double x, double y) {
    const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
                 C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
                 C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
    double z = x * x;
    double r = z * (C1 + z * (C2 + z * (C3 + z * (C4 + z * (C5 + z * C6)))));
    double ax = __builtin_fabs(x);
    if (ax < 0.3) return 1.0 - (0.5 * z - (z * r - x * y));
    double qx;
    if (ax > 0.78125) {
        qx = 0.28125;
    } else {
        unsigned long long b = (unsigned long long)__double_as_longlong(ax);
        b = (b - 0x0020000000000000ULL) & 0xFFFFFFFF00000000ULL;
        qx = __longlong_as_double((long long)b);
    }
    double hz = 0.5 * z - qx;
    double a = 1.0 - qx;
    return a - (hz - (z * r - x * y));
}
__device__ __forceinline__ int exp_bits(double x) {
    return (int)(((unsigned long long)__double_as_longlong(x) >> 52) & 0x7ff);
}
__device__ inline double rt_sin(double x) {
    const double ax = __builtin_fabs(x);
    if (ax <= 0.78539816339744828) return k_sin_y(x, 0.0);
    if (!(ax < 823549.6)) return ::sin(x);
    const double invpio2 = 6.36619772367581382433e-01, pio2_1 = 1.57079632673412561417e+00,
                 pio2_1t = 6.07710050650619224932e-11, pio2_2 = 6.07710050630396597660e-11,
                 pio2_2t = 2.02226624879595063154e-21, pio2_3 = 2.02226624871116645580e-21,
                 pio2_3t = 8.47842766036889956997e-32;
    const int n = (int)(ax * invpio2 + 0.5);
    const double fn = (double)n;
    double r = ax - fn * pio2_1;
    double w = fn * pio2_1t;
    double y0 = r - w;
    const int j = exp_bits(ax);
    if (j - exp_bits(y0) > 16) {
        double t = r;
        w = fn * pio2_2;
        r = t - w;
        w = fn * pio2_2t - ((t - r) - w);
        y0 = r - w;
        if (j - exp_bits(y0) > 49) {
            t = r;
            w = fn * pio2_3;
            r = t - w;
            w = fn * pio2_3t - ((t - r) - w);
            y0 = r - w;
        }
    }
    double y1 = (r - y0) - w;
    int q = n;
    if (x < 0.0) {
        y0 = -y0;
        y1 = -y1;
        q = -n;
    }
    switch (q & 3) {
        case 0: return k_sin_y(y0, y1);
        case 1: return k_cos_y(y0, y1);
        case 2: return -k_sin_y(y0, y1);
        default: return -k_cos_y(y0, y1);
    }
}
__device__ __forceinline__ float rt_sin(float x) { return ::sinf(x); }

__device__ __forceinline__ double floor_(double x) { return __builtin_floor(x); }
__device__ __forceinline__ float floor_(float x) { return __builtin_floorf(x); }
__device__ __forceinline__ double trunc_(double x) { return __builtin_trunc(x); }
__device__ __forceinline__ float trunc_(float x) { return __builtin_truncf(x); }

// f64::rem_euclid(256.) then `as usize` of an integral value (a floor plus 0
// or 1): x mod 256 in two's complement; non-finite -> NaN -> 0; values too
// large for the integer type are multiples of 256 -> 0.
__device__ __forceinline__ uint32_t perlin_index(double x) {
    return __builtin_fabs(x) < 9.2e18 ? (uint32_t)((long long)x & 255) : 0u;
}
__device__ __forceinline__ uint32_t perlin_index(float x) {
    return __builtin_fabsf(x) < 2147483648.f ? (uint32_t)((int)x & 255) : 0u;   // beyond: multiples of 256
}

// Sphere::get_sphere_uv, sphere.rs:49-54 (the library atan2 / acos: the f64
// results may differ from libm's in the last ulp, which moves a checker edge
// only for points within an ulp of it)
__device__ __forceinline__ void sphere_uv(V3<double> n, double& u, double& v) {
    u = ::atan2(-n.z, n.x) / P<double>::kTau;
    v = ::acos(n.y) / P<double>::kPi;
}
__device__ __forceinline__ void sphere_uv(V3<float> n, float& u, float& v) {
    u = ::atan2f(-n.z, n.x) * 0.159154943091895335769f;
    v = ::acosf(n.y) * P<float>::kInvPi;
}

}  // namespace dev
}  // namespace rtw
