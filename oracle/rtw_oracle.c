/*
 * rtw_oracle.c -- CPU restatement (f64) of the reference's hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see rtw_oracle.h).  Every function cites the
 * reference file:line it restates; paths are relative to the reference root
 * (N9199/ray_tracing_weekend).  Build: oracle/Makefile (gcc, -ffp-contract=off
 * so that every a*b+c rounds twice, as in the reference's Rust code).
 *
 * Deliberate, documented deviations from the reference (none changes the
 * sampled distribution):
 *  - RNG: the reference seeds a SmallRng per pixel from thread_rng
 *    (camera.rs:346), so its stream is unobtainable.  Here every (pixel,
 *    sample) pair gets its own xoshiro256++ stream (rand 0.8.6's SmallRng
 *    algorithm on 64-bit targets) seeded through splitmix64 from
 *    (seed, pixel, sample).  The distributions on top of it restate rand
 *    0.8.6's published algorithms (Standard, Open01, Uniform::new_inclusive,
 *    gen_range's widening multiply) in the reference's draw order, except
 *    for two draws that cannot change any sampled law: the light pick is one
 *    gen_index(n) (choose()'s reservoir step adds a gen_index(1)), and
 *    UnitSphere does not shuffle its three i.i.d. coordinates.
 *  - cos/sin of 2*pi*r are evaluated by rtwo_sincos_2pi (fdlibm kernel
 *    polynomials after an exact quadrant reduction of r) instead of libm's
 *    cos(2*PI*r); both are within ~1 ulp of the true value.  The GPU f64 path
 *    evaluates the same polynomial, which is what makes bit-level parity
 *    possible.
 *  - Sphere/plane UVs (atan2/acos, sphere.rs:49-54; plane.rs:181-194) are
 *    not computed: only textures read them and every in-scope material uses
 *    SolidColour (texture.rs:15-22), so the output does not depend on them.
 */
#include "rtw_oracle.h"

#include <float.h>
#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#define PI 3.14159265358979323846
#define TAU (2.0 * PI)

/* ------------------------------------------------------------------------ */
/* Vec3 (geometry/src/vec3/vec.rs)                                          */
/* ------------------------------------------------------------------------ */
typedef struct { double x, y, z; } v3;

static inline v3 mk(double x, double y, double z) { v3 r = {x, y, z}; return r; }
static inline v3 ld(const double *p) { return mk(p[0], p[1], p[2]); }
static inline void st3(double *p, v3 v) { p[0] = v.x; p[1] = v.y; p[2] = v.z; }
static inline v3 add(v3 a, v3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }      /* vec.rs:151-157 */
static inline v3 sub(v3 a, v3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }      /* vec.rs:166-172 */
static inline v3 neg(v3 a) { return mk(-a.x, -a.y, -a.z); }                            /* vec.rs:175-180 */
static inline v3 muls(v3 a, double s) { return mk(a.x * s, a.y * s, a.z * s); }       /* vec.rs:209-214 */
static inline v3 divs(v3 a, double s) { return mk(a.x / s, a.y / s, a.z / s); }       /* vec.rs:217-222 */
static inline v3 mulv(v3 a, v3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }     /* vec.rs:132-138 */
static inline double dot(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }    /* vec.rs:70-72 */
static inline v3 cross(v3 a, v3 b) {                                                   /* vec.rs:76-82 */
    return mk(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
static inline double length(v3 a) { return sqrt(dot(a, a)); }                         /* vec.rs:58-66 */
static inline v3 normalize(v3 a) { return divs(a, length(a)); }                       /* vec.rs:86-94 */
static inline int near_zero(v3 a) {                                                    /* vec.rs:98-101 */
    const double e = 1e-8;
    return fabs(a.x) < e && fabs(a.y) < e && fabs(a.z) < e;
}
static inline v3 reflect(v3 v, v3 n) {                                                 /* vec.rs:105-107 */
    return sub(v, muls(muls(n, 2.0), dot(v, n)));
}
static inline v3 refract(v3 v, v3 n, double eta) {                                     /* vec.rs:111-116 */
    double cos_theta = fmin(dot(v, neg(n)), 1.0);
    v3 perp = muls(add(v, muls(n, cos_theta)), eta);
    v3 par = muls(n, -(sqrt(1.0 - dot(perp, perp))));
    return add(perp, par);
}
static inline v3 at(v3 o, v3 d, double t) { return add(o, muls(d, t)); }               /* ray.rs:25-27 */

/* Onb (geometry/src/onb.rs:8-35) */
typedef struct { v3 u, v, w; } onb_t;
static inline onb_t onb_new(v3 n) {
    onb_t b;
    b.w = normalize(n);
    v3 a = fabs(b.w.x) > 0.9 ? mk(0.0, 1.0, 0.0) : mk(1.0, 0.0, 0.0);
    b.v = normalize(cross(b.w, a));
    b.u = cross(b.w, b.v);
    return b;
}
static inline v3 onb_transform(onb_t b, v3 x) {
    /* (0..3).map(|i| e[i] * x[i]).sum(): fold from Vec3::default() (vec.rs:283-287) */
    v3 acc = mk(0.0, 0.0, 0.0);
    acc = add(acc, muls(b.u, x.x));
    acc = add(acc, muls(b.v, x.y));
    acc = add(acc, muls(b.w, x.z));
    return acc;
}

/* ------------------------------------------------------------------------ */
/* sin/cos of 2*pi*r (stands in for phi = 2*PI*r; phi.cos(), phi.sin()      */
/* at utils.rs:155-157 and sphere.rs:123-125).                              */
/* ------------------------------------------------------------------------ */
static double k_sin(double x) {
    const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
                 S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
                 S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
    double z = x * x;
    double v = z * x;
    double r = S2 + z * (S3 + z * (S4 + z * (S5 + z * S6)));
    return x + v * (S1 + z * r);
}
static double k_cos(double x) {
    const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
                 C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
                 C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
    double z = x * x;
    double r = z * (C1 + z * (C2 + z * (C3 + z * (C4 + z * (C5 + z * C6)))));
    double ax = fabs(x);
    if (ax < 0.3) return 1.0 - (0.5 * z - (z * r));
    double qx;
    if (ax > 0.78125) {
        qx = 0.28125;
    } else {
        uint64_t bits;
        memcpy(&bits, &ax, 8);
        bits = (bits - 0x0020000000000000ULL) & 0xFFFFFFFF00000000ULL;
        memcpy(&qx, &bits, 8);
    }
    double hz = 0.5 * z - qx;
    double a = 1.0 - qx;
    return a - (hz - z * r);
}
void rtwo_sincos_2pi(double r, double *s, double *c) {
    double q = rint(r * 4.0);
    double f = r - q * 0.25;          /* exact: |f| <= 1/8 */
    double x = f * TAU;
    double ks = k_sin(x), kc = k_cos(x);
    switch (((int64_t)q) & 3) {
    case 0: *s = ks; *c = kc; break;
    case 1: *s = kc; *c = -ks; break;
    case 2: *s = -ks; *c = -kc; break;
    default: *s = -kc; *c = ks; break;
    }
}

/* ------------------------------------------------------------------------ */
/* RNG: xoshiro256++ (SmallRng, rand 0.8.6 on 64-bit) + splitmix64 seeding  */
/* ------------------------------------------------------------------------ */
static inline uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
static inline uint64_t splitmix_next(uint64_t *x) {
    *x += 0x9E3779B97F4A7C15ULL;
    return mix64(*x);
}
static inline uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }

void rtwo_rng_seed(uint64_t seed, uint64_t pixel_index, uint64_t sample_index, uint64_t st[4]) {
    uint64_t k = mix64(seed + 0x9E3779B97F4A7C15ULL * (pixel_index + 1));
    k = mix64(k ^ (0xD1B54A32D192ED03ULL * (sample_index + 1)));
    /* Xoshiro256PlusPlus::seed_from_u64: fill the state from a SplitMix64 stream */
    for (int i = 0; i < 4; ++i) st[i] = splitmix_next(&k);
}
uint64_t rtwo_rng_next(uint64_t s[4]) {
    uint64_t result = rotl(s[0] + s[3], 23) + s[0];
    uint64_t t = s[1] << 17;
    s[2] ^= s[0];
    s[3] ^= s[1];
    s[1] ^= s[2];
    s[0] ^= s[3];
    s[2] ^= t;
    s[3] = rotl(s[3], 45);
    return result;
}
static inline double bits_to_unit12(uint64_t v) {
    /* into_float_with_exponent(0) of (v >> 12): a double in [1, 2) */
    uint64_t b = (v >> 12) | 0x3FF0000000000000ULL;
    double d;
    memcpy(&d, &b, 8);
    return d;
}
/* rand 0.8.6 Standard for f64: (v >> 11) * 2^-53, in [0, 1) */
double rtwo_rand_std(uint64_t st[4]) {
    return (1.0 / 9007199254740992.0) * (double)(rtwo_rng_next(st) >> 11);
}
/* rand 0.8.6 Open01 for f64: 52-bit fraction, (0, 1) */
double rtwo_rand_open01(uint64_t st[4]) {
    return bits_to_unit12(rtwo_rng_next(st)) - (1.0 - DBL_EPSILON / 2.0);
}
/* rand 0.8.6 UniformFloat::new_inclusive(low, high) scale */
static double uniform_incl_scale(double low, double high) {
    double max_rand = bits_to_unit12(~0ULL) - 1.0;   /* 1 - 2^-52 */
    double scale = (high - low) / max_rand;
    while (scale * max_rand + low > high) {
        uint64_t b;
        memcpy(&b, &scale, 8);
        b -= 1;
        memcpy(&scale, &b, 8);
    }
    return scale;
}
static inline double uniform_sample(uint64_t st[4], double low, double scale) {
    double v01 = bits_to_unit12(rtwo_rng_next(st)) - 1.0;
    return v01 * scale + low;
}
double rtwo_rand_uniform_incl(uint64_t st[4], double low, double high) {
    return uniform_sample(st, low, uniform_incl_scale(low, high));
}
/* gen_index / gen_range(0..n) for u32 (rand 0.8.6 UniformInt::
 * sample_single_inclusive with the leading-zeros zone), next_u32 = next_u64>>32 */
uint32_t rtwo_rand_index(uint64_t st[4], uint32_t n) {
    uint32_t range = n;
    uint32_t zone = (range << __builtin_clz(range)) - 1u;
    for (;;) {
        uint32_t v = (uint32_t)(rtwo_rng_next(st) >> 32);
        uint64_t m = (uint64_t)v * (uint64_t)range;
        uint32_t hi = (uint32_t)(m >> 32), lo = (uint32_t)m;
        if (lo <= zone) return hi;
    }
}

/* ------------------------------------------------------------------------ */
/* Random utilities (shared/src/utils.rs:93-161)                            */
/* ------------------------------------------------------------------------ */
/* UnitSphere, utils.rs:99-122: rejection sampling in the cube [-1, 1)^3.  The
 * reference shuffles the three i.i.d. coordinates before the test
 * (utils.rs:116, two gen_index draws); a permutation of i.i.d. coordinates
 * does not change their joint law, so the build draws no shuffle indices. */
static v3 unit_sphere(uint64_t st[4]) {
    for (;;) {
        double in[3];
        for (int k = 0; k < 3; ++k) in[k] = 2.0 * rtwo_rand_std(st) - 1.0;
        v3 out = mk(in[0], in[1], in[2]);
        if (dot(out, out) < 1.0) return out;
    }
}
static v3 unit_disk(uint64_t st[4]) {                                         /* utils.rs:124-144 */
    for (;;) {
        double x = 2.0 * rtwo_rand_std(st) - 1.0;
        double z = 2.0 * rtwo_rand_std(st) - 1.0;
        v3 out = mk(x, 0.0, z);
        if (dot(out, out) < 1.0) return out;
    }
}
static v3 cosine_hemisphere(uint64_t st[4]) {                                 /* utils.rs:146-161 */
    double r1 = rtwo_rand_std(st);
    double r2 = rtwo_rand_std(st);
    double s, c;
    rtwo_sincos_2pi(r1, &s, &c);
    double sq = sqrt(r2);
    return mk(c * sq, s * sq, sqrt(1.0 - r2));
}
void rtwo_unit_sphere(uint64_t st[4], double out[3]) { st3(out, unit_sphere(st)); }
void rtwo_cosine_hemisphere(uint64_t st[4], double out[3]) { st3(out, cosine_hemisphere(st)); }

/* ------------------------------------------------------------------------ */
/* Primitives                                                               */
/* ------------------------------------------------------------------------ */
/* Sphere::hit, sphere.rs:61-80 -- root selection only */
static inline int sphere_t(v3 c, double radius, v3 o, v3 d, double tmin, double tmax, double *t) {
    v3 oc = sub(o, c);
    double a = dot(d, d);
    double half_b = dot(d, oc);
    double cc = dot(oc, oc) - radius * radius;
    double disc = half_b * half_b - a * cc;
    if (!(disc > 0.0)) return 0;
    double sq = sqrt(disc);
    double root = (-half_b - sq) / a;
    if (!(tmin <= root && root <= tmax)) {
        root = (-half_b + sq) / a;
        if (!(tmin <= root && root <= tmax)) return 0;
    }
    *t = root;
    return 1;
}
/* HitRecord::new, hittable.rs:101-129 (+ outward normal sphere.rs:82-83) */
typedef struct { v3 p, normal; double t; int front; uint32_t mat; } hitrec;
static inline void make_record(v3 o, v3 d, double t, v3 outward, uint32_t mat, hitrec *rec) {
    rec->p = at(o, d, t);
    rec->front = dot(d, outward) < 0.0;
    rec->normal = rec->front ? outward : neg(outward);
    rec->t = t;
    rec->mat = mat;
}
static inline void sphere_record(v3 c, double radius, v3 o, v3 d, double t, uint32_t mat, hitrec *rec) {
    v3 p = at(o, d, t);
    v3 outward = divs(sub(p, c), radius);
    make_record(o, d, t, outward, mat, rec);
}
int rtwo_sphere_hit(const double sph[4], const double o[3], const double d[3],
                    double tmin, double tmax, double *t, double normal[3], int *front) {
    double tt;
    if (!sphere_t(ld(sph), sph[3], ld(o), ld(d), tmin, tmax, &tt)) return 0;
    hitrec rec;
    sphere_record(ld(sph), sph[3], ld(o), ld(d), tt, 0, &rec);
    *t = tt;
    st3(normal, rec.normal);
    *front = rec.front;
    return 1;
}
/* Plane::hit, plane.rs:61-76 (one-sided: only rays moving along +n) */
static inline int plane_t(v3 p0, v3 n, v3 o, v3 d, double tmin, double tmax, double *t) {
    double denom = dot(d, n);
    if (!(denom > DBL_EPSILON)) return 0;
    double tt = -(dot(sub(o, p0), n) / denom);
    if (!(tmin <= tt && tt <= tmax)) return 0;
    *t = tt;
    return 1;
}
int rtwo_plane_hit(const double pl[6], const double o[3], const double d[3],
                   double tmin, double tmax, double *t, double normal[3], int *front) {
    double tt;
    if (!plane_t(ld(pl), ld(pl + 3), ld(o), ld(d), tmin, tmax, &tt)) return 0;
    hitrec rec;
    make_record(ld(o), ld(d), tt, ld(pl + 3), 0, &rec);
    *t = tt;
    st3(normal, rec.normal);
    *front = rec.front;
    return 1;
}

/* AABBox slab test, hittable.rs:291-339 */
typedef struct { double mn[3], mx[3]; } aabb;
static inline int aabb_hit(const aabb *b, v3 o, v3 d, double rs, double re) {
    double ox[3] = {o.x, o.y, o.z}, dx[3] = {d.x, d.y, d.z};
    double t0 = (b->mn[0] - ox[0]) / dx[0];
    double t1 = (b->mx[0] - ox[0]) / dx[0];
    if (signbit(dx[0])) { double tmp = t0; t0 = t1; t1 = tmp; }
    double tmin = t0, tmax = t1;
    for (int k = 1; k < 3; ++k) {
        double a0 = (b->mn[k] - ox[k]) / dx[k];
        double a1 = (b->mx[k] - ox[k]) / dx[k];
        if (signbit(dx[k])) { double tmp = a0; a0 = a1; a1 = tmp; }
        if (tmax < a0 || tmin > a1) return 0;
        tmin = fmax(tmin, a0);   /* f64::max: NaN-ignoring, like fmax */
        tmax = fmin(tmax, a1);
    }
    return fmax(rs, tmin) <= fmin(re, tmax);
}
int rtwo_aabb_hit(const double box[6], const double o[3], const double d[3],
                  double tmin, double tmax) {
    aabb b;
    memcpy(b.mn, box, 24);
    memcpy(b.mx, box + 3, 24);
    return aabb_hit(&b, ld(o), ld(d), tmin, tmax);
}
/* AABBox::pad_to_minimum + enclose_aabbox, aabox.rs:129-175 */
static void aabb_enclose(aabb *a, const aabb *b) {
    for (int k = 0; k < 3; ++k) {
        a->mn[k] = fmin(a->mn[k], b->mn[k]);
        a->mx[k] = fmax(a->mx[k], b->mx[k]);
    }
    const double delta = 0.0001;
    for (int k = 0; k < 3; ++k) {
        if (a->mx[k] - a->mn[k] < delta) { a->mn[k] -= delta; a->mx[k] += delta; }
    }
}

/* ------------------------------------------------------------------------ */
/* Quad (quadrilateral.rs)                                                  */
/* ------------------------------------------------------------------------ */
typedef struct { v3 q, u, v, w, normal; double area; aabb box; } rquad;

/* Quad::new, quadrilateral.rs:37-56 */
static rquad quad_new(const double *p) {
    rquad Q;
    Q.q = ld(p);
    Q.u = ld(p + 3);
    Q.v = ld(p + 6);
    /* AABBox::from_points([q + (u + v) * 0.5, q, q + v, q + u, q + u + v]):
     * the first point, then enclose (with pad_to_minimum) each of the rest */
    v3 pts[5] = {add(Q.q, muls(add(Q.u, Q.v), 0.5)), Q.q, add(Q.q, Q.v), add(Q.q, Q.u),
                 add(add(Q.q, Q.u), Q.v)};
    Q.box.mn[0] = Q.box.mx[0] = pts[0].x;
    Q.box.mn[1] = Q.box.mx[1] = pts[0].y;
    Q.box.mn[2] = Q.box.mx[2] = pts[0].z;
    for (int i = 1; i < 5; ++i) {
        aabb pb = {{pts[i].x, pts[i].y, pts[i].z}, {pts[i].x, pts[i].y, pts[i].z}};
        aabb_enclose(&Q.box, &pb);
    }
    v3 n = cross(Q.u, Q.v);
    Q.w = divs(n, dot(n, n));                  /* normal / normal.square_length() */
    Q.area = length(n);
    Q.normal = divs(n, Q.area);
    return Q;
}

/* Quad::hit, quadrilateral.rs:79-100 (+ get_quad_uv :58-63) */
static inline int quad_hit_t(const rquad *Q, v3 o, v3 d, double tmin, double tmax, double *t) {
    double denom = dot(d, Q->normal);
    if (!(fabs(denom) > DBL_EPSILON)) return 0;
    double tt = -(dot(sub(o, Q->q), Q->normal) / denom);
    if (!(tt >= tmin && tt <= tmax)) return 0;
    v3 pq = sub(at(o, d, tt), Q->q);
    double alpha = dot(cross(pq, Q->v), Q->w);
    double beta = dot(cross(Q->u, pq), Q->w);
    if (!(alpha >= 0.0 && alpha <= 1.0 && beta >= 0.0 && beta <= 1.0)) return 0;
    *t = tt;
    return 1;
}

/* Quad::pdf_value, quadrilateral.rs:102-112 */
static double quad_pdf_value(const rquad *Q, v3 o, v3 d) {
    double t;
    if (!quad_hit_t(Q, o, d, 0.0, INFINITY, &t)) return 0.0;
    v3 n = dot(d, Q->normal) < 0.0 ? Q->normal : neg(Q->normal);   /* HitRecord::new */
    double distance_squared = t * t * dot(d, d);
    double cosine = fabs(dot(d, n) / length(d));
    return distance_squared / (cosine * Q->area);
}

/* Quad::random, quadrilateral.rs:114-118 */
static v3 quad_random(const rquad *Q, v3 o, uint64_t st[4]) {
    double r1 = rtwo_rand_open01(st);
    double r2 = rtwo_rand_open01(st);
    v3 p = add(add(Q->q, muls(Q->u, r1)), muls(Q->v, r2));
    return sub(p, o);
}

int rtwo_quad_hit(const double quad[9], const double o[3], const double d[3],
                  double tmin, double tmax, double out[6]) {
    rquad Q = quad_new(quad);
    double t;
    if (!quad_hit_t(&Q, ld(o), ld(d), tmin, tmax, &t)) return 0;
    v3 pq = sub(at(ld(o), ld(d), t), Q.q);
    out[0] = t;
    out[1] = dot(cross(pq, Q.v), Q.w);
    out[2] = dot(cross(Q.u, pq), Q.w);
    st3(out + 3, dot(ld(d), Q.normal) < 0.0 ? Q.normal : neg(Q.normal));
    return 1;
}
double rtwo_quad_pdf_value(const double quad[9], const double o[3], const double d[3]) {
    rquad Q = quad_new(quad);
    return quad_pdf_value(&Q, ld(o), ld(d));
}
void rtwo_quad_random(const double quad[9], const double o[3], uint64_t st[4], double out[3]) {
    rquad Q = quad_new(quad);
    st3(out, quad_random(&Q, ld(o), st));
}
void rtwo_quad_aabb(const double quad[9], double box[6]) {
    rquad Q = quad_new(quad);
    memcpy(box, Q.box.mn, 24);
    memcpy(box + 3, Q.box.mx, 24);
}

/* ------------------------------------------------------------------------ */
/* Transformed<Cuboid>                                                      */
/* ------------------------------------------------------------------------ */
typedef struct { double m[3][3]; } mat3;
/* Mul<Vec3> for Matrix3 (matrix3.rs:94-105): each row . p */
static inline v3 mat3_mul(const mat3 *M, v3 p) {
    return mk(dot(ld(M->m[0]), p), dot(ld(M->m[1]), p), dot(ld(M->m[2]), p));
}
typedef struct {
    rquad quads[6];             /* the cuboid's quads, object space */
    mat3 R, Ri;                 /* Transformation.rotation and its inverse */
    v3 T, Ti;                   /* translation, -(Ri T) */
    int invertible;
    aabb box;                   /* Transformed::get_aabbox, world space */
} rbox;

static rbox box_new(const double *b) {
    rbox B;
    /* Cuboid::new, cuboid.rs:26-47: the (padded) box of p and q */
    aabb ab = {{b[0], b[1], b[2]}, {b[0], b[1], b[2]}};
    aabb qb = {{b[3], b[4], b[5]}, {b[3], b[4], b[5]}};
    aabb_enclose(&ab, &qb);
    v3 mn = mk(ab.mn[0], ab.mn[1], ab.mn[2]), mx = mk(ab.mx[0], ab.mx[1], ab.mx[2]);
    v3 delta = sub(mx, mn);
    v3 dx = mk(delta.x, 0.0, 0.0), dy = mk(0.0, delta.y, 0.0), dz = mk(0.0, 0.0, delta.z);
    v3 args[6][3] = {{mn, dx, dy}, {mn, dy, dz}, {mn, dx, dz},
                     {mx, neg(dx), neg(dy)}, {mx, neg(dy), neg(dz)}, {mx, neg(dx), neg(dz)}};
    for (int i = 0; i < 6; ++i) {
        double q[9];
        st3(q, args[i][0]);
        st3(q + 3, args[i][1]);
        st3(q + 6, args[i][2]);
        B.quads[i] = quad_new(q);
    }
    /* Cuboid::get_aabbox (cuboid.rs:61-71): fold of the quads' boxes */
    aabb cub = B.quads[0].box;
    for (int i = 1; i < 6; ++i) aabb_enclose(&cub, &B.quads[i].box);
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) B.R.m[r][c] = b[6 + 3 * r + c];
    B.T = ld(b + 15);
    /* Transformed::get_aabbox: from_points(instance box corners (get_points
     * order, aabox.rs:113-124) mapped through transform_point3d) */
    const double *lo = cub.mn, *hi = cub.mx;
    v3 corners[8] = {mk(lo[0], lo[1], lo[2]), mk(lo[0], hi[1], lo[2]), mk(lo[0], lo[1], hi[2]),
                     mk(lo[0], hi[1], hi[2]), mk(hi[0], lo[1], lo[2]), mk(hi[0], hi[1], lo[2]),
                     mk(hi[0], lo[1], hi[2]), mk(hi[0], hi[1], hi[2])};
    for (int i = 0; i < 8; ++i) {
        v3 w = add(mat3_mul(&B.R, corners[i]), B.T);
        if (i == 0) {
            B.box.mn[0] = B.box.mx[0] = w.x;
            B.box.mn[1] = B.box.mx[1] = w.y;
            B.box.mn[2] = B.box.mx[2] = w.z;
        } else {
            aabb pb = {{w.x, w.y, w.z}, {w.x, w.y, w.z}};
            aabb_enclose(&B.box, &pb);
        }
    }
    /* Matrix3::inverse (matrix3.rs:9-28) and Transformation::inverse */
    const double a = B.R.m[0][0], bb = B.R.m[0][1], c = B.R.m[0][2];
    const double d = B.R.m[1][0], e = B.R.m[1][1], f = B.R.m[1][2];
    const double g = B.R.m[2][0], h = B.R.m[2][1], i = B.R.m[2][2];
    const double det = a * (e * i - f * h) + bb * (f * g - d * i) + c * (d * h - e * g);
    B.invertible = isnormal(det);
    const double A = e * i - f * h, Bc = f * g - d * i, C = d * h - e * g;
    const double D = c * h - bb * i, E = a * i - c * g, F = bb * g - a * h;
    const double G = bb * f - c * e, H = c * d - a * f, I = a * e - bb * d;
    B.Ri.m[0][0] = A / det; B.Ri.m[0][1] = D / det; B.Ri.m[0][2] = G / det;
    B.Ri.m[1][0] = Bc / det; B.Ri.m[1][1] = E / det; B.Ri.m[1][2] = H / det;
    B.Ri.m[2][0] = C / det; B.Ri.m[2][1] = F / det; B.Ri.m[2][2] = I / det;
    B.Ti = neg(mat3_mul(&B.Ri, B.T));
    return B;
}

/* Transformed<Cuboid>::hit (entities/transformations.rs:14-29 over
 * Cuboid::hit, cuboid.rs:50-58).  The ray goes to object space through the
 * inverse: origin by transform_point3d, direction by transform_vector3d --
 * which in geometry/src/transformations.rs:112-114 also ADDS the translation
 * (the reference's behaviour, kept).  Closest of the six quads (min_by: the
 * first minimum), then only the hit point goes back to world space; the
 * normal stays in object space. */
static int box_hit(const rbox *B, v3 o, v3 d, double tmin, double tmax, double *t, v3 *pw, v3 *nrm,
                   int *front) {
    if (!B->invertible) return 0;
    v3 o2 = add(mat3_mul(&B->Ri, o), B->Ti);
    v3 d2 = add(mat3_mul(&B->Ri, d), B->Ti);
    int best = -1;
    double bt = INFINITY;
    for (int k = 0; k < 6; ++k) {
        double tt;
        if (quad_hit_t(&B->quads[k], o2, d2, tmin, tmax, &tt) && (best < 0 || tt < bt)) {
            bt = tt;
            best = k;
        }
    }
    if (best < 0) return 0;
    *t = bt;
    if (pw) {
        v3 n = B->quads[best].normal;
        *front = dot(d2, n) < 0.0;                               /* HitRecord::new */
        *nrm = *front ? n : neg(n);
        *pw = add(mat3_mul(&B->R, at(o2, d2, bt)), B->T);        /* transform_point3d */
    }
    return 1;
}

int rtwo_box_hit(const double box[18], const double o[3], const double d[3],
                 double tmin, double tmax, double out[8]) {
    rbox B = box_new(box);
    double t;
    v3 pw, n;
    int front;
    if (!box_hit(&B, ld(o), ld(d), tmin, tmax, &t, &pw, &n, &front)) return 0;
    out[0] = t;
    st3(out + 1, pw);
    st3(out + 4, n);
    out[7] = front;
    return 1;
}
void rtwo_box_aabb(const double box[18], double aabb_out[6]) {
    rbox B = box_new(box);
    memcpy(aabb_out, B.box.mn, 24);
    memcpy(aabb_out + 3, B.box.mx, 24);
}

/* Sphere::pdf_value, sphere.rs:101-111 */
static inline double sphere_pdf_value(v3 c, double radius, v3 o, v3 d) {
    double t;
    if (!sphere_t(c, radius, o, d, 0.0, INFINITY, &t)) return 0.0;
    double dist2 = dot(sub(c, o), sub(c, o));
    double cos_theta_max = sqrt(1.0 - radius * radius / dist2);
    double solid_angle = TAU * (1.0 - cos_theta_max);
    return 1.0 / solid_angle;
}
double rtwo_sphere_pdf_value(const double sph[4], const double o[3], const double d[3]) {
    return sphere_pdf_value(ld(sph), sph[3], ld(o), ld(d));
}
/* Sphere::random, sphere.rs:114-127 */
static inline v3 sphere_random(v3 c, double radius, v3 o, uint64_t st[4]) {
    v3 direction = sub(c, o);
    double distance = length(direction);
    onb_t uvw = onb_new(direction);
    double r1 = rtwo_rand_std(st);
    double r2 = rtwo_rand_std(st);
    double z = 1.0 + r1 * (sqrt(1.0 - radius * radius / (distance * distance)) - 1.0);
    double s, cph;
    rtwo_sincos_2pi(r2, &s, &cph);
    double x = cph * sqrt(1.0 - z * z);
    double y = s * sqrt(1.0 - z * z);
    return onb_transform(uvw, mk(x, y, z));
}
void rtwo_sphere_random(const double sph[4], const double o[3], uint64_t st[4], double out[3]) {
    st3(out, sphere_random(ld(sph), sph[3], ld(o), st));
}
void rtwo_onb(const double n[3], double u[3], double v[3], double w[3]) {
    onb_t b = onb_new(ld(n));
    st3(u, b.u); st3(v, b.v); st3(w, b.w);
}
/* Dialectric::reflectance, material.rs:450-454 ((1-c).powi(5) = x*((x*x)*(x*x))) */
double rtwo_reflectance(double cosine, double ref_idx) {
    double r0 = (1.0 - ref_idx) / (1.0 + ref_idx);
    r0 = r0 * r0;
    double x = 1.0 - cosine;
    double x2 = x * x;
    double p5 = x * (x2 * x2);
    return r0 + (1.0 - r0) * p5;
}
void rtwo_reflect(const double v[3], const double n[3], double out[3]) { st3(out, reflect(ld(v), ld(n))); }
void rtwo_refract(const double v[3], const double n[3], double eta, double out[3]) {
    st3(out, refract(ld(v), ld(n), eta));
}

/* ------------------------------------------------------------------------ */
/* Reference BVH restatement (bvh.rs:106-188; hittable_list.rs:270-406)     */
/* ------------------------------------------------------------------------ */
/* Object ids: planes, quads, spheres (three "type groups", as the          */
/* TypeId-sorted RawHittableVecs of a HittableList).                        */
#define NG 4
typedef struct {
    int leaf;
    int left, right;            /* node children */
    /* leaf: up to two groups, each a list of object ids */
    int group_start[NG], group_len[NG];
    aabb group_box[NG];
    aabb box;                   /* leaf: HittableList.aabbox; node: cached enclose */
} bvh_node;

typedef struct {
    const rtwo_scene *sc;
    aabb *obj_box;              /* per object */
    int *obj_ids;               /* storage of leaf groups */
    int n_ids;
    bvh_node *nodes;
    int n_nodes, cap_nodes;
    int root;
    int max_depth;
} bvh_t;

/* object ids: [0, n_planes) planes, then n_quads quads, n_boxes boxes, then the spheres */
static inline int box_base(const rtwo_scene *sc) { return (int)(sc->n_planes + sc->n_quads); }
static inline int sphere_base(const rtwo_scene *sc) { return (int)(sc->n_planes + sc->n_quads + sc->n_boxes); }

static aabb object_box(const rtwo_scene *sc, int id) {
    aabb b;
    if (id >= (int)sc->n_planes && id < box_base(sc)) {
        rquad Q = quad_new(sc->quads + 9 * (id - (int)sc->n_planes));
        return Q.box;
    }
    if (id >= box_base(sc) && id < sphere_base(sc)) {
        rbox B = box_new(sc->boxes + 18 * (id - box_base(sc)));
        return B.box;
    }
    if (id < (int)sc->n_planes) {
        /* Plane::get_aabbox, plane.rs:218-242 */
        const double *n = sc->planes + 6 * id + 3;
        double e = DBL_EPSILON;
        int flat_x = fabs(n[2]) < e && fabs(n[1]) < e;
        int flat_y = fabs(n[0]) < e && fabs(n[2]) < e;
        int flat_z = fabs(n[0]) < e && fabs(n[1]) < e;
        b.mn[0] = flat_x ? 0.0 : -INFINITY; b.mx[0] = flat_x ? 0.0 : INFINITY;
        b.mn[1] = flat_y ? 0.0 : -INFINITY; b.mx[1] = flat_y ? 0.0 : INFINITY;
        b.mn[2] = flat_z ? 0.0 : -INFINITY; b.mx[2] = flat_z ? 0.0 : INFINITY;
    } else {
        /* Sphere::new aabox, sphere.rs:42-45 */
        const double *s = sc->spheres + 4 * (id - sphere_base(sc));
        for (int k = 0; k < 3; ++k) { b.mn[k] = s[k] - s[3]; b.mx[k] = s[k] + s[3]; }
    }
    return b;
}

static int new_node(bvh_t *t) {
    if (t->n_nodes == t->cap_nodes) {
        t->cap_nodes = t->cap_nodes ? 2 * t->cap_nodes : 64;
        t->nodes = (bvh_node *)realloc(t->nodes, sizeof(bvh_node) * t->cap_nodes);
    }
    memset(&t->nodes[t->n_nodes], 0, sizeof(bvh_node));
    return t->n_nodes++;
}

/* A HittableList being split: its two type groups (planes, spheres), each an
 * ordered list of ids in the group's Vec order. */
typedef struct { int *ids[NG]; int len[NG]; } hlist;

static int hl_len(const hlist *h) { return h->len[0] + h->len[1] + h->len[2] + h->len[3]; }

static aabb group_box(const bvh_t *t, const int *ids, int len) {
    /* Slice::get_aabbox: reduce(|acc, e| acc.enclose(e)) (utils.rs:152-158) */
    aabb b = t->obj_box[ids[0]];
    for (int k = 1; k < len; ++k) aabb_enclose(&b, &t->obj_box[ids[k]]);
    return b;
}

static int cmp_dbl_total(double a, double b) {
    /* f64::total_cmp restricted to the values that occur (no NaN boxes) */
    if (a < b) return -1;
    if (a > b) return 1;
    if (signbit(a) && !signbit(b)) return -1;
    if (!signbit(a) && signbit(b)) return 1;
    return 0;
}
typedef struct { double s, e; } range_t;
static int cmp_range(const void *pa, const void *pb) {
    const range_t *a = (const range_t *)pa, *b = (const range_t *)pb;
    int c = cmp_dbl_total(a->s, b->s);
    return c ? c : cmp_dbl_total(a->e, b->e);
}

static int build(bvh_t *t, hlist *h, int depth) {
    if (depth > t->max_depth) t->max_depth = depth;
    int len = hl_len(h);
    int node = new_node(t);
    if (len <= 5) {
        bvh_node *nd = &t->nodes[node];
        nd->leaf = 1;
        int have = 0;
        for (int g = 0; g < NG; ++g) {
            nd->group_start[g] = t->n_ids;
            nd->group_len[g] = h->len[g];
            if (h->len[g]) {
                memcpy(t->obj_ids + t->n_ids, h->ids[g], sizeof(int) * h->len[g]);
                nd->group_box[g] = group_box(t, h->ids[g], h->len[g]);
                if (!have) { nd->box = nd->group_box[g]; have = 1; }
                else aabb_enclose(&nd->box, &nd->group_box[g]);
                t->n_ids += h->len[g];
            }
        }
        return node;
    }
    /* best_split, hittable_list.rs:318-379 */
    size_t best_imb = (size_t)-1;
    double best_size = INFINITY, best_coord = 0.0;
    int best_axis = 0;
    range_t *tmp = (range_t *)malloc(sizeof(range_t) * len);
    for (int axis = 0; axis < 3; ++axis) {
        int m = 0;
        for (int g = 0; g < NG; ++g)
            for (int k = 0; k < h->len[g]; ++k) {
                aabb b = t->obj_box[h->ids[g][k]];
                tmp[m].s = b.mn[axis]; tmp[m].e = b.mx[axis]; ++m;
            }
        qsort(tmp, len, sizeof(range_t), cmp_range);   /* sort_by is stable; equal keys are identical */
        double pivot = tmp[len / 2].s;
        int pp = 0;
        while (pp < len && cmp_dbl_total(tmp[pp].s, pivot) < 0) ++pp;
        double size = tmp[len - 1].e - tmp[0].s;
        size_t imb = (size_t)(len - 2 * pp);
        /* (best.0, -best.1) > (imb, -size) */
        int better = (best_imb > imb) || (best_imb == imb && (-best_size > -size));
        if (better) { best_imb = imb; best_size = size; best_axis = axis; best_coord = pivot; }
    }
    free(tmp);
    /* split_by (hittable_list.rs:296-316, raw.rs:84-104): pop from the back,
     * start > coord goes "right"; best_split hands back (right, left). */
    hlist parts[2];
    for (int p = 0; p < 2; ++p)
        for (int g = 0; g < NG; ++g) {
            parts[p].ids[g] = (int *)malloc(sizeof(int) * (h->len[g] + 1));
            parts[p].len[g] = 0;
        }
    for (int g = 0; g < NG; ++g)
        for (int k = h->len[g] - 1; k >= 0; --k) {
            int id = h->ids[g][k];
            int right = t->obj_box[id].mn[best_axis] > best_coord;
            hlist *dst = &parts[right ? 0 : 1];   /* parts[0] = geometric right = BVH "left" */
            dst->ids[g][dst->len[g]++] = id;
        }
    int result;
    if (hl_len(&parts[0]) == len || hl_len(&parts[1]) == len) {
        /* bvh.rs:127-130: degenerate split becomes a (large) leaf */
        hlist *all = hl_len(&parts[0]) == len ? &parts[0] : &parts[1];
        bvh_node *nd = &t->nodes[node];
        nd->leaf = 1;
        int have = 0;
        for (int g = 0; g < NG; ++g) {
            nd->group_start[g] = t->n_ids;
            nd->group_len[g] = all->len[g];
            if (all->len[g]) {
                memcpy(t->obj_ids + t->n_ids, all->ids[g], sizeof(int) * all->len[g]);
                nd->group_box[g] = group_box(t, all->ids[g], all->len[g]);
                if (!have) { nd->box = nd->group_box[g]; have = 1; }
                else aabb_enclose(&nd->box, &nd->group_box[g]);
                t->n_ids += all->len[g];
            }
        }
        result = node;
    } else {
        int l = build(t, &parts[0], depth + 1);
        int r = build(t, &parts[1], depth + 1);
        bvh_node *nd = &t->nodes[node];
        nd->leaf = 0;
        nd->left = l;
        nd->right = r;
        nd->box = t->nodes[l].box;
        aabb_enclose(&nd->box, &t->nodes[r].box);
        result = node;
    }
    for (int p = 0; p < 2; ++p)
        for (int g = 0; g < NG; ++g) free(parts[p].ids[g]);
    return result;
}

static void bvh_build(bvh_t *t, const rtwo_scene *sc) {
    memset(t, 0, sizeof(*t));
    t->sc = sc;
    int n = (int)(sc->n_planes + sc->n_quads + sc->n_boxes + sc->n_spheres);
    t->obj_box = (aabb *)malloc(sizeof(aabb) * (n ? n : 1));
    t->obj_ids = (int *)malloc(sizeof(int) * (n ? n : 1));
    for (int i = 0; i < n; ++i) t->obj_box[i] = object_box(sc, i);
    hlist h;
    h.len[0] = (int)sc->n_planes;
    h.len[1] = (int)sc->n_quads;
    h.len[2] = (int)sc->n_boxes;
    h.len[3] = (int)sc->n_spheres;
    int first = 0;
    for (int g = 0; g < NG; ++g) {
        h.ids[g] = (int *)malloc(sizeof(int) * (h.len[g] + 1));
        for (int i = 0; i < h.len[g]; ++i) h.ids[g][i] = first + i;
        first += h.len[g];
    }
    t->root = build(t, &h, 1);
    for (int g = 0; g < NG; ++g) free(h.ids[g]);
}
static void bvh_free(bvh_t *t) {
    free(t->obj_box);
    free(t->obj_ids);
    free(t->nodes);
}
/* Bounded for BoundedVolumeHierarchy (bvh.rs:147-152): recomputed per call */
static aabb node_box_recomputed(const bvh_t *t, int node) {
    const bvh_node *nd = &t->nodes[node];
    if (nd->leaf) return nd->box;
    aabb b = node_box_recomputed(t, nd->left);
    aabb r = node_box_recomputed(t, nd->right);
    aabb_enclose(&b, &r);
    return b;
}

typedef struct { double t; int id; } cand;

static inline int object_hit_t(const rtwo_scene *sc, int id, v3 o, v3 d, double tmin, double tmax, double *t) {
    if (id < (int)sc->n_planes) {
        const double *p = sc->planes + 6 * id;
        return plane_t(ld(p), ld(p + 3), o, d, tmin, tmax, t);
    }
    if (id < box_base(sc)) {
        rquad Q = quad_new(sc->quads + 9 * (id - (int)sc->n_planes));
        return quad_hit_t(&Q, o, d, tmin, tmax, t);
    }
    if (id < sphere_base(sc)) {
        rbox B = box_new(sc->boxes + 18 * (id - box_base(sc)));
        return box_hit(&B, o, d, tmin, tmax, t, NULL, NULL, NULL);
    }
    const double *s = sc->spheres + 4 * (id - sphere_base(sc));
    return sphere_t(ld(s), s[3], o, d, tmin, tmax, t);
}

/* BoundedVolumeHierarchy::hit, bvh.rs:164-188 */
static cand bvh_hit(const bvh_t *t, int node, v3 o, v3 d, double tmin, double tmax, int recompute) {
    const bvh_node *nd = &t->nodes[node];
    cand best = {INFINITY, -1};
    if (nd->leaf) {
        /* HittableList::hit (hittable_list.rs:395-406) over the type groups,
         * each group bounded_hit (group AABB) then Slice::hit (utils.rs:172-179) */
        for (int g = 0; g < NG; ++g) {
            if (!nd->group_len[g]) continue;
            if (!aabb_hit(&nd->group_box[g], o, d, tmin, tmax)) continue;
            for (int k = 0; k < nd->group_len[g]; ++k) {
                int id = t->obj_ids[nd->group_start[g] + k];
                if (!aabb_hit(&t->obj_box[id], o, d, tmin, tmax)) continue;
                double tt;
                if (object_hit_t(t->sc, id, o, d, tmin, tmax, &tt) && (best.id < 0 || tt < best.t)) {
                    best.t = tt; best.id = id;
                }
            }
        }
        return best;
    }
    aabb lb = recompute ? node_box_recomputed(t, nd->left) : t->nodes[nd->left].box;
    cand a = {INFINITY, -1}, b = {INFINITY, -1};
    if (aabb_hit(&lb, o, d, tmin, tmax)) a = bvh_hit(t, nd->left, o, d, tmin, tmax, recompute);
    aabb rb = recompute ? node_box_recomputed(t, nd->right) : t->nodes[nd->right].box;
    if (aabb_hit(&rb, o, d, tmin, tmax)) b = bvh_hit(t, nd->right, o, d, tmin, tmax, recompute);
    if (a.id < 0) return b;
    if (b.id < 0) return a;
    return b.t < a.t ? b : a;   /* min_by: first minimum wins */
}

int rtwo_bvh_stats(const rtwo_scene *sc, uint32_t *nodes, uint32_t *leaves, uint32_t *depth) {
    bvh_t t;
    bvh_build(&t, sc);
    uint32_t nl = 0;
    for (int i = 0; i < t.n_nodes; ++i) nl += t.nodes[i].leaf;
    *nodes = (uint32_t)t.n_nodes;
    *leaves = nl;
    *depth = (uint32_t)t.max_depth;
    bvh_free(&t);
    return 0;
}

/* ------------------------------------------------------------------------ */
/* The render loop                                                          */
/* ------------------------------------------------------------------------ */
typedef struct {
    const rtwo_camera *cam;
    const rtwo_scene *sc;
    const bvh_t *bvh;
    int accel;
    uint64_t seed;
    double u_scale;             /* Uniform::new_inclusive(-0.5, 0.5) scale */
    double *path;               /* debugging: per-segment {o, d, id, t} or NULL */
    uint32_t path_cap;
} ctx_t;

/* world.hit(&r, EPSILON..=INFINITY), closest over every primitive */
static int world_hit_id(const ctx_t *cx, v3 o, v3 d, hitrec *rec, int *id_out) {
    const rtwo_scene *sc = cx->sc;
    const double tmin = DBL_EPSILON, tmax = INFINITY;
    int best = -1;
    double bt = INFINITY;
    if (cx->accel == RTWO_ACCEL_BRUTE) {
        /* Every object is reached through bounded_hit (hittable.rs:190-196,
         * utils.rs:172-179): its own AABB test comes first.  That matters for
         * a plane, whose AABB pins the normal axis at coordinate 0 wherever
         * the plane lies (plane.rs:218-242), and for a negative-radius sphere,
         * whose AABB is inverted and never hit (sphere.rs:42-45).  For a
         * positive-radius sphere the box contains the sphere, so the test is
         * skipped (it can only disagree on rounding at the silhouette). */
        for (uint32_t k = 0; k < sc->n_planes; ++k) {
            double t;
            aabb pb = object_box(sc, (int)k);
            if (aabb_hit(&pb, o, d, tmin, tmax) &&
                plane_t(ld(sc->planes + 6 * k), ld(sc->planes + 6 * k + 3), o, d, tmin, tmax, &t) &&
                (best < 0 || t < bt)) { bt = t; best = (int)k; }
        }
        for (uint32_t k = 0; k < sc->n_quads; ++k) {
            /* a quad's AABB (points enclosed, thin axes padded) holds the quad */
            rquad Q = quad_new(sc->quads + 9 * k);
            double t;
            if (aabb_hit(&Q.box, o, d, tmin, tmax) && quad_hit_t(&Q, o, d, tmin, tmax, &t) &&
                (best < 0 || t < bt)) { bt = t; best = (int)(sc->n_planes + k); }
        }
        for (uint32_t k = 0; k < sc->n_boxes; ++k) {
            rbox B = box_new(sc->boxes + 18 * k);
            double t;
            if (aabb_hit(&B.box, o, d, tmin, tmax) && box_hit(&B, o, d, tmin, tmax, &t, NULL, NULL, NULL) &&
                (best < 0 || t < bt)) { bt = t; best = box_base(sc) + (int)k; }
        }
        for (uint32_t k = 0; k < sc->n_spheres; ++k) {
            const double *s = sc->spheres + 4 * k;
            double t;
            if (s[3] < 0.0) continue;
            if (sphere_t(ld(s), s[3], o, d, tmin, tmax, &t) && (best < 0 || t < bt)) {
                bt = t; best = sphere_base(sc) + (int)k;
            }
        }
    } else {
        cand c = bvh_hit(cx->bvh, cx->bvh->root, o, d, tmin, tmax, cx->accel == RTWO_ACCEL_BVH_REF);
        best = c.id;
        bt = c.t;
    }
    if (id_out) *id_out = best;
    if (best < 0) return 0;
    if (best < (int)sc->n_planes) {
        make_record(o, d, bt, ld(sc->planes + 6 * best + 3), sc->plane_mat[best], rec);
    } else if (best < box_base(sc)) {
        uint32_t k = (uint32_t)best - sc->n_planes;
        rquad Q = quad_new(sc->quads + 9 * k);
        make_record(o, d, bt, Q.normal, sc->quad_mat[k], rec);
    } else if (best < sphere_base(sc)) {
        uint32_t k = (uint32_t)(best - box_base(sc));
        rbox B = box_new(sc->boxes + 18 * k);
        double t2;
        box_hit(&B, o, d, DBL_EPSILON, INFINITY, &t2, &rec->p, &rec->normal, &rec->front);
        rec->t = bt;
        rec->mat = sc->box_mat[k];
    } else {
        uint32_t k = (uint32_t)(best - sphere_base(sc));
        const double *s = sc->spheres + 4 * k;
        sphere_record(ld(s), s[3], o, d, bt, sc->sphere_mat[k], rec);
    }
    return 1;
}

/* The light list in list order: entry k is sphere light_index(k) or quad. */
static inline uint32_t n_light_list(const rtwo_scene *sc) { return sc->n_lights + sc->n_light_quads; }
static inline void light_entry(const rtwo_scene *sc, uint32_t k, int *is_quad, uint32_t *idx) {
    if (!sc->light_kinds) {
        *is_quad = k >= sc->n_lights;
        *idx = *is_quad ? k - sc->n_lights : k;
        return;
    }
    uint32_t ns = 0, nq = 0;
    for (uint32_t i = 0; i < k; ++i) {
        if (sc->light_kinds[i]) ++nq;
        else ++ns;
    }
    *is_quad = sc->light_kinds[k] != 0;
    *idx = *is_quad ? nq : ns;
}

/* world.hit for one ray (KATs / debugging): returns the object id (planes,
 * quads, boxes, spheres numbering) or -1; out = {t, p xyz, normal xyz, front}. */
int rtwo_world_hit(const rtwo_scene *sc, int accel, const double o[3], const double d[3], double out[8]) {
    bvh_t bvh;
    int use_bvh = accel != RTWO_ACCEL_BRUTE;
    if (use_bvh) bvh_build(&bvh, sc);
    ctx_t cx = {NULL, sc, use_bvh ? &bvh : NULL, accel, 0, 0.0, NULL, 0};
    hitrec rec;
    int id = -1;
    if (world_hit_id(&cx, ld(o), ld(d), &rec, &id)) {
        out[0] = rec.t;
        st3(out + 1, rec.p);
        st3(out + 4, rec.normal);
        out[7] = rec.front;
    }
    if (use_bvh) bvh_free(&bvh);
    return id;
}

/* HittableList::pdf_value, hittable_list.rs:408-412 */
static double lights_pdf_value(const rtwo_scene *sc, v3 o, v3 d) {
    double acc = 0.0;
    const uint32_t n = n_light_list(sc);
    uint32_t ns = 0, nq = 0;
    for (uint32_t k = 0; k < n; ++k) {
        int is_quad = sc->light_kinds ? sc->light_kinds[k] != 0 : k >= sc->n_lights;
        if (is_quad) {
            rquad Q = quad_new(sc->light_quads + 9 * nq++);
            acc = acc + quad_pdf_value(&Q, o, d);
        } else {
            const double *s = sc->lights + 4 * ns++;
            acc = acc + sphere_pdf_value(ld(s), s[3], o, d);
        }
    }
    return acc / (double)n;
}
/* HittableList::random, hittable_list.rs:414-419: iter_hittable().choose(rng)
 * picks a light uniformly, then its random().  rand 0.8.6's
 * IteratorRandom::choose reaches that uniform pick through a reservoir step
 * over the flat_map (an extra gen_index(1) draw, then gen_index(n)); the build
 * draws the uniform index directly with one gen_index(n). */
static v3 lights_random(const rtwo_scene *sc, v3 o, uint64_t st[4]) {
    const uint32_t pick = rtwo_rand_index(st, n_light_list(sc));
    int is_quad;
    uint32_t idx;
    light_entry(sc, pick, &is_quad, &idx);
    if (is_quad) {
        rquad Q = quad_new(sc->light_quads + 9 * idx);
        return quad_random(&Q, o, st);
    }
    const double *s = sc->lights + 4 * idx;
    return sphere_random(ld(s), s[3], o, st);
}

/* Camera::get_ray, camera.rs:274-293 */
static void get_ray(const ctx_t *cx, uint32_t i, uint32_t j, uint64_t st[4], v3 *o, v3 *d) {
    const rtwo_camera *c = cx->cam;
    double ox = uniform_sample(st, -0.5, cx->u_scale);
    double oy = uniform_sample(st, -0.5, cx->u_scale);
    v3 ps = add(add(ld(c->pixel00_loc), muls(ld(c->pixel_delta_u), (double)i + ox)),
                muls(ld(c->pixel_delta_v), (double)j + oy));
    v3 origin;
    if (c->defocus_angle <= DBL_EPSILON) {
        origin = ld(c->center);
    } else {
        v3 p = unit_disk(st);
        origin = add(add(ld(c->center), muls(ld(c->defocus_disk_u), p.x)), muls(ld(c->defocus_disk_v), p.z));
    }
    *o = origin;
    *d = sub(ps, origin);
}

/* ray_colour_call + ray_colour_tail_call, camera.rs:439-522, as a loop */
static v3 trace(const ctx_t *cx, uint32_t i, uint32_t j, uint32_t s, rtwo_stats *stats) {
    const rtwo_camera *c = cx->cam;
    const rtwo_scene *sc = cx->sc;
    uint64_t st[4];
    rtwo_rng_seed(cx->seed, (uint64_t)j * c->image_width + i, s, st);
    v3 o, d;
    get_ray(cx, i, j, st, &o, &d);
    v3 mult = mk(1.0, 1.0, 1.0);
    v3 res = mk(0.0, 0.0, 0.0);
    const v3 zero = mk(0.0, 0.0, 0.0);
    uint32_t depth = c->max_depth;
    for (;;) {
        if (depth == 0) return add(zero, res);                     /* :470-472 */
        hitrec rec;
        const uint64_t seg = stats->segments++;
        int hid = -1;
        const int hit = world_hit_id(cx, o, d, &rec, &hid);
        if (cx->path && seg < cx->path_cap) {
            double *e = cx->path + 8 * seg;
            st3(e, o);
            st3(e + 3, d);
            e[6] = hid;
            e[7] = hit ? rec.t : INFINITY;
        }
        if (!hit)
            return add(mulv(mult, ld(c->background)), res);        /* :473-475 */
        const uint32_t m = rec.mat;
        const double *mp = sc->mat_params + 5 * m;
        /* :480-482: DiffuseLight::emitted = its colour (material.rs:508-514);
         * every other material emits black (material.rs:42-44) */
        const v3 emitted = sc->mat_type[m] == RTWO_DIFFUSE_LIGHT ? ld(mp) : zero;
        switch (sc->mat_type[m]) {
        case RTWO_METAL: {                                          /* material.rs:407-421 */
            v3 refl = reflect(normalize(d), rec.normal);
            v3 dir = add(refl, muls(unit_sphere(st), mp[3]));
            if (!(dot(dir, rec.normal) > 0.0)) return add(mulv(mult, emitted), res);
            mult = mulv(mult, ld(mp));                              /* Reflect: :488-500 */
            o = rec.p; d = dir;
            break;
        }
        case RTWO_DIELECTRIC: {                                     /* material.rs:458-487 */
            double ratio = rec.front ? 1.0 / mp[4] : mp[4];
            v3 unit = normalize(d);
            double cos_t = fmin(dot(unit, neg(rec.normal)), 1.0);
            double sin_t = sqrt(1.0 - cos_t * cos_t);
            int cannot = ratio * sin_t > 1.0;
            v3 dir;
            if (cannot || rtwo_reflectance(cos_t, ratio) > rtwo_rand_open01(st))
                dir = reflect(unit, rec.normal);
            else
                dir = refract(unit, rec.normal, ratio);
            mult = mulv(mult, mk(1.0, 1.0, 1.0));
            o = rec.p; d = dir;
            break;
        }
        case RTWO_LAMBERTIAN: {                                     /* material.rs:357-376 */
            stats->lambertian++;
            v3 att = ld(mp);
            onb_t uvw = onb_new(rec.normal);                        /* CosinePdf::new, pdf.rs:38-42 */
            v3 dir;
            if (rtwo_rand_std(st) < 0.5)                            /* MixturePdf::generate pdf.rs:94-100 */
                dir = lights_random(sc, rec.p, st);
            else
                dir = onb_transform(uvw, cosine_hemisphere(st));
            double cos_w = dot(normalize(dir), uvw.w) / PI;         /* CosinePdf::value pdf.rs:45-48 */
            double pdf = lights_pdf_value(sc, rec.p, dir) * 0.5 + fmax(cos_w, 0.0) * 0.5;
            double spdf = fmax(dot(rec.normal, normalize(dir)) / PI, 0.0);
            v3 w = divs(muls(att, spdf), pdf);
            v3 new_mult = mulv(mult, w);                            /* :518 */
            res = add(res, mulv(mult, emitted));                    /* :519 */
            mult = new_mult;
            o = rec.p; d = dir;
            break;
        }
        default:                      /* Invisible, DiffuseLight: scatter None (:484-486) */
            return add(mulv(mult, emitted), res);
        }
        depth -= 1;
    }
}

void rtwo_trace_sample(const rtwo_camera *cam, const rtwo_scene *sc, uint64_t seed,
                       uint32_t i, uint32_t j, uint32_t s, double out_rgb[3], rtwo_stats *stats) {
    rtwo_trace_path(cam, sc, seed, i, j, s, RTWO_ACCEL_BRUTE, out_rgb, stats, NULL, 0);
}

uint32_t rtwo_trace_path(const rtwo_camera *cam, const rtwo_scene *sc, uint64_t seed, uint32_t i, uint32_t j,
                         uint32_t s, int accel, double out_rgb[3], rtwo_stats *stats, double *path,
                         uint32_t path_cap) {
    bvh_t bvh;
    const int use_bvh = accel != RTWO_ACCEL_BRUTE;
    if (use_bvh) bvh_build(&bvh, sc);
    ctx_t cx = {cam, sc, use_bvh ? &bvh : NULL, accel, seed, uniform_incl_scale(-0.5, 0.5), path, path_cap};
    rtwo_stats local = {0, 0, 0, 0};
    v3 c = trace(&cx, i, j, s, &local);
    if (use_bvh) bvh_free(&bvh);
    st3(out_rgb, c);
    if (stats) {
        stats->samples += 1;
        stats->segments += local.segments;
        stats->lambertian += local.lambertian;
        stats->nan_samples += (c.x != c.x || c.y != c.y || c.z != c.z);
    }
    return (uint32_t)local.segments;
}

typedef struct {
    const ctx_t *cx;
    uint32_t chunk;
    uint32_t row_begin, row_end, row_step, col_begin, col_end;
    double *out;
    volatile uint32_t *next_row;   /* shared work counter (row index into the row list) */
    uint32_t n_rows;
    rtwo_stats stats;
    char pad[64];               /* keep workers' stats on separate cache lines */
} worker_t;

static void *worker(void *arg) {
    worker_t *w = (worker_t *)arg;
    const ctx_t *cx = w->cx;
    const uint32_t W = cx->cam->image_width, spp = cx->cam->samples_per_pixel;
    rtwo_stats local = {0, 0, 0, 0};
    for (;;) {
        uint32_t r = __atomic_fetch_add(w->next_row, 1u, __ATOMIC_RELAXED);
        if (r >= w->n_rows) break;
        uint32_t j = w->row_begin + r * w->row_step;
        for (uint32_t i = w->col_begin; i < w->col_end; ++i) {
            v3 total = mk(0.0, 0.0, 0.0);
            for (uint32_t s0 = 0; s0 < spp; s0 += w->chunk) {
                uint32_t s1 = s0 + w->chunk < spp ? s0 + w->chunk : spp;
                v3 part = mk(0.0, 0.0, 0.0);          /* fold(Colour::default(), +) */
                for (uint32_t s = s0; s < s1; ++s) {
                    v3 c = trace(cx, i, j, s, &local);
                    local.samples++;
                    local.nan_samples += (c.x != c.x || c.y != c.y || c.z != c.z);
                    part = add(part, c);
                }
                total = add(total, part);
            }
            st3(w->out + ((size_t)j * W + i) * 3, total);
        }
    }
    w->stats = local;
    return NULL;
}

static int has_lambertian(const rtwo_scene *sc) {
    for (uint32_t k = 0; k < sc->n_materials; ++k)
        if (sc->mat_type[k] == RTWO_LAMBERTIAN) return 1;
    return 0;
}

int rtwo_render(const rtwo_camera *cam, const rtwo_scene *sc, uint64_t seed,
                uint32_t chunk, int accel, int nthreads,
                uint32_t row_begin, uint32_t row_end, uint32_t row_step,
                uint32_t col_begin, uint32_t col_end,
                double *out, rtwo_stats *stats) {
    if (!cam || !sc || !out) return -1;
    if (has_lambertian(sc) && n_light_list(sc) == 0) return -1;
    if (row_step == 0) row_step = 1;
    if (row_end > cam->image_height) row_end = cam->image_height;
    if (col_end > cam->image_width) col_end = cam->image_width;
    if (chunk == 0 || chunk > cam->samples_per_pixel) chunk = cam->samples_per_pixel ? cam->samples_per_pixel : 1;
    if (nthreads < 1) nthreads = 1;
    bvh_t bvh;
    int use_bvh = accel != RTWO_ACCEL_BRUTE;
    if (use_bvh) bvh_build(&bvh, sc);
    ctx_t cx = {cam, sc, use_bvh ? &bvh : NULL, accel, seed, uniform_incl_scale(-0.5, 0.5), NULL, 0};
    uint32_t n_rows = row_begin < row_end ? (row_end - row_begin + row_step - 1) / row_step : 0;
    volatile uint32_t next_row = 0;
    worker_t *ws = (worker_t *)calloc((size_t)nthreads, sizeof(worker_t));
    pthread_t *th = (pthread_t *)calloc((size_t)nthreads, sizeof(pthread_t));
    for (int k = 0; k < nthreads; ++k) {
        ws[k].cx = &cx; ws[k].chunk = chunk;
        ws[k].row_begin = row_begin; ws[k].row_end = row_end; ws[k].row_step = row_step;
        ws[k].col_begin = col_begin; ws[k].col_end = col_end;
        ws[k].out = out; ws[k].next_row = &next_row; ws[k].n_rows = n_rows;
    }
    for (int k = 1; k < nthreads; ++k) pthread_create(&th[k], NULL, worker, &ws[k]);
    worker(&ws[0]);
    for (int k = 1; k < nthreads; ++k) pthread_join(th[k], NULL);
    if (stats) {
        memset(stats, 0, sizeof(*stats));
        for (int k = 0; k < nthreads; ++k) {
            stats->samples += ws[k].stats.samples;
            stats->segments += ws[k].stats.segments;
            stats->lambertian += ws[k].stats.lambertian;
            stats->nan_samples += ws[k].stats.nan_samples;
        }
    }
    free(ws);
    free(th);
    if (use_bvh) bvh_free(&bvh);
    return 0;
}

/* ------------------------------------------------------------------------ */
/* CameraBuilder::build, camera.rs:114-218                                   */
/* ------------------------------------------------------------------------ */
static uint32_t round_u32(double x) {
    /* f64::round (half away from zero) then `as u32` (saturating, NaN -> 0) */
    double r = round(x);
    if (!(r > 0.0)) return 0;
    if (r >= 4294967295.0) return 4294967295u;
    return (uint32_t)r;
}
int rtwo_camera_build(const rtwo_camera_builder *b, rtwo_camera *out) {
    double aspect;
    uint32_t H, W;
    int ha = b->has_aspect_ratio, hh = b->has_image_height, hw = b->has_image_width;
    if (!ha && !hh && !hw) { aspect = 1.0; H = 100; W = 100; }
    else if (!ha && !hh && hw) { aspect = 1.0; H = b->image_width; W = b->image_width; }
    else if (!ha && hh && !hw) { aspect = 1.0; H = b->image_height; W = b->image_height; }
    else if (ha && !hh && !hw) { aspect = b->aspect_ratio; H = round_u32(100.0 / b->aspect_ratio); W = 100; }
    else if (!ha && hh && hw) { aspect = (double)b->image_width / (double)b->image_height; H = b->image_height; W = b->image_width; }
    else if (ha && !hh && hw) { aspect = b->aspect_ratio; H = round_u32((double)b->image_width / b->aspect_ratio); W = b->image_width; }
    else if (ha && hh && !hw) { aspect = b->aspect_ratio; H = b->image_height; W = round_u32((double)b->image_height * b->aspect_ratio); }
    else { aspect = b->aspect_ratio; H = b->image_height; W = b->image_width; }

    v3 center = ld(b->lookfrom);
    double theta = b->vfov * (PI / 180.0);                          /* f64::to_radians */
    double h = tan(theta / 2.0);
    double vh = 2.0 * h * b->focus_dist;
    double vw = vh * aspect;
    v3 w = sub(ld(b->lookfrom), ld(b->lookat));
    if (near_zero(cross(ld(b->vup), w))) w = add(w, mk(0.1, 0.0, 0.0));
    w = normalize(w);
    v3 u = normalize(cross(ld(b->vup), w));
    v3 v = cross(w, u);
    v3 vu = muls(u, vw), vv = muls(v, vh);
    v3 du = divs(vu, (double)W), dv = divs(vv, (double)H);
    v3 ul = sub(sub(sub(center, muls(w, b->focus_dist)), divs(vu, 2.0)), divs(vv, 2.0));
    v3 p00 = add(ul, divs(add(du, dv), 2.0));
    double rad = tan(b->defocus_angle / 2.0) * b->focus_dist;
    memset(out, 0, sizeof(*out));
    out->image_width = W;
    out->image_height = H;
    out->samples_per_pixel = b->samples_per_pixel;
    out->max_depth = b->max_depth;
    memcpy(out->background, b->background, 24);
    out->defocus_angle = b->defocus_angle;
    st3(out->center, center);
    st3(out->pixel00_loc, p00);
    st3(out->pixel_delta_u, du);
    st3(out->pixel_delta_v, dv);
    st3(out->defocus_disk_u, muls(u, rad));
    st3(out->defocus_disk_v, muls(v, rad));
    return 0;
}

/* ------------------------------------------------------------------------ */
/* scenes::simple, scenes/src/lib.rs:155-233                                 */
/* ------------------------------------------------------------------------ */
int rtwo_scene_simple(uint64_t seed, int n,
                      uint32_t max_spheres, double *spheres, uint32_t *sphere_mat,
                      uint32_t *n_spheres,
                      double *planes, uint32_t *plane_mat, uint32_t *n_planes,
                      uint32_t max_mats, uint32_t *mat_type, double *mat_params,
                      uint32_t *n_mats,
                      uint32_t max_lights, double *lights, uint32_t *n_lights) {
    uint64_t st[4];
    uint64_t k = seed;
    for (int q = 0; q < 4; ++q) st[q] = splitmix_next(&k);   /* SmallRng::seed_from_u64 */
    uint32_t ns = 0, nm = 0, nl = 0;
#define PUSH_MAT(type, r, g, b, fuzz, ior)                                     \
    do {                                                                       \
        if (nm >= max_mats) return -1;                                         \
        mat_type[nm] = (type);                                                 \
        mat_params[5 * nm + 0] = (r); mat_params[5 * nm + 1] = (g);            \
        mat_params[5 * nm + 2] = (b); mat_params[5 * nm + 3] = (fuzz);        \
        mat_params[5 * nm + 4] = (ior);                                        \
        ++nm;                                                                  \
    } while (0)
#define PUSH_SPHERE(x, y, z, rad, mat)                                         \
    do {                                                                       \
        if (ns >= max_spheres) return -1;                                      \
        spheres[4 * ns + 0] = (x); spheres[4 * ns + 1] = (y);                  \
        spheres[4 * ns + 2] = (z); spheres[4 * ns + 3] = (rad);                \
        sphere_mat[ns] = (mat);                                                \
        ++ns;                                                                  \
    } while (0)
#define PUSH_LIGHT(x, y, z, rad)                                               \
    do {                                                                       \
        if (nl >= max_lights) return -1;                                       \
        lights[4 * nl + 0] = (x); lights[4 * nl + 1] = (y);                    \
        lights[4 * nl + 2] = (z); lights[4 * nl + 3] = (rad);                  \
        ++nl;                                                                  \
    } while (0)

    /* ground: Plane((0,0,0), (0,1,0), Lambertian(0.9)) :163-169 */
    PUSH_MAT(RTWO_LAMBERTIAN, 0.9, 0.9, 0.9, 0.0, 0.0);
    v3 pn = normalize(mk(0.0, 1.0, 0.0));
    planes[0] = 0.0; planes[1] = 0.0; planes[2] = 0.0;
    planes[3] = pn.x; planes[4] = pn.y; planes[5] = pn.z;
    plane_mat[0] = 0;
    *n_planes = 1;
    const double ui_scale = uniform_incl_scale(0.5, 1.0);   /* random_f64_2, utils.rs:94-97 */
    for (int a = -n; a < n; ++a) {
        for (int b = -n; b < n; ++b) {
            double choose_mat = rtwo_rand_std(st);
            double cx = (double)a + 0.9 * rtwo_rand_std(st);
            double cz = (double)b + 0.9 * rtwo_rand_std(st);
            v3 c = mk(cx, 0.2, cz);
            if (length(sub(c, mk(4.0, 0.2, 0.0))) > 0.9) {
                if (choose_mat < 0.8) {
                    double a1 = rtwo_rand_std(st), a2 = rtwo_rand_std(st), a3 = rtwo_rand_std(st);
                    double b1 = rtwo_rand_std(st), b2 = rtwo_rand_std(st), b3 = rtwo_rand_std(st);
                    PUSH_MAT(RTWO_LAMBERTIAN, a1 * b1, a2 * b2, a3 * b3, 0.0, 0.0);
                } else if (choose_mat < 0.95) {
                    double r = uniform_sample(st, 0.5, ui_scale);
                    double g = uniform_sample(st, 0.5, ui_scale);
                    double bb = uniform_sample(st, 0.5, ui_scale);
                    double fuzz = 1.0 - uniform_sample(st, 0.5, ui_scale);
                    PUSH_MAT(RTWO_METAL, r, g, bb, fuzz, 0.0);
                } else {
                    PUSH_LIGHT(cx, 0.2, cz, 0.2);
                    PUSH_MAT(RTWO_DIELECTRIC, 1.0, 1.0, 1.0, 0.0, 1.5);
                }
                PUSH_SPHERE(cx, 0.2, cz, 0.2, nm - 1);
            }
        }
    }
    /* :210-217 */
    PUSH_MAT(RTWO_DIELECTRIC, 1.0, 1.0, 1.0, 0.0, 1.5);
    PUSH_SPHERE(0.0, 1.0, 0.0, 1.0, nm - 1);
    PUSH_MAT(RTWO_LAMBERTIAN, 0.4, 0.2, 0.1, 0.0, 0.0);
    PUSH_SPHERE(-4.0, 1.0, 0.0, 1.0, nm - 1);
    PUSH_MAT(RTWO_METAL, 0.7, 0.6, 0.5, 0.0, 0.0);
    PUSH_SPHERE(4.0, 1.0, 0.0, 1.0, nm - 1);
    PUSH_LIGHT(0.0, 1.0, 0.0, 1.0);
#undef PUSH_MAT
#undef PUSH_SPHERE
#undef PUSH_LIGHT
    *n_spheres = ns;
    *n_mats = nm;
    *n_lights = nl;
    return 0;
}
