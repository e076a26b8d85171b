// bvh4_check.cpp -- host-only check of the 4-wide octant BVH (host/bvh.cpp
// collapse_bvh4) and of the traversal the kernel runs on it, restated on the
// CPU in f32: for random rays the closest sphere must equal brute force.
//   g++ -O2 -std=c++17 -I ray_tracing_weekend_amd/csrc tools/bvh4_check.cpp \
//       ray_tracing_weekend_amd/csrc/host/bvh.cpp -o /tmp/bvh4_check && /tmp/bvh4_check
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <random>
#include <vector>

#include "host/bvh.hpp"

using rtw::Bvh4Build;
using rtw::BvhBuild;

static int fails = 0;
#define CHECK(c, ...)                  \
    do {                               \
        if (!(c)) {                    \
            printf("FAIL: " __VA_ARGS__); \
            printf("\n");              \
            ++fails;                   \
        }                              \
    } while (0)

struct Node4 {   // octant copy, as staged by capi.cpp
    float nx[4], ny[4], nz[4], fx[4], fy[4], fz[4];
    int32_t child[4];
};

static float down(double x) {
    float r = (float)x;
    return (double)r > x ? nextafterf(r, -INFINITY) : r;
}
static float up(double x) {
    float r = (float)x;
    return (double)r < x ? nextafterf(r, INFINITY) : r;
}

int main(int argc, char** argv) {
    const uint32_t n = argc > 1 ? (uint32_t)atoi(argv[1]) : 484;
    std::mt19937_64 g(7);
    std::uniform_real_distribution<double> U(-11, 11), R(0.05, 0.3);
    std::vector<double> sph(4 * n);
    for (uint32_t k = 0; k < n; ++k) {
        sph[4 * k] = U(g);
        sph[4 * k + 1] = k % 7 == 0 ? 1.0 : 0.2;
        sph[4 * k + 2] = U(g);
        sph[4 * k + 3] = k % 7 == 0 ? 1.0 : R(g);
    }
    const BvhBuild bb = rtw::build_bvh(sph.data(), n, 1e-5);
    const Bvh4Build b4 = rtw::collapse_bvh4(bb);
    printf("n=%u binary nodes=%zu depth=%u | bvh4 nodes=%zu depth=%u max_stack=%u\n", n, bb.nodes.size(),
           bb.depth, b4.nodes.size(), b4.depth, b4.max_stack);
    // structure: every leaf sphere reached once, orders are permutations
    std::vector<int> seen(n, 0);
    double fill = 0;
    for (const auto& nd : b4.nodes) {
        CHECK(nd.n >= 1 && nd.n <= 4 || n == 0, "node fill %u", nd.n);
        fill += nd.n;
        for (int o = 0; o < 8; ++o) {
            int mask = 0;
            for (uint32_t q = 0; q < nd.n; ++q) mask |= 1 << nd.order[o][q];
            CHECK(mask == (1 << nd.n) - 1, "order not a permutation");
        }
        for (uint32_t q = 0; q < nd.n; ++q)
            if (nd.child[q] < 0) {
                const uint32_t code = ~(uint32_t)nd.child[q];
                for (uint32_t k = 0; k < (code & 15u); ++k) seen[bb.order[(code >> 4) + k]]++;
            }
    }
    printf("average children per node %.2f\n", fill / std::max<size_t>(1, b4.nodes.size()));
    for (uint32_t k = 0; k < n; ++k) CHECK(seen[k] == 1, "sphere %u seen %d times", k, seen[k]);
    // stage the octant copies exactly like capi.cpp
    const size_t n4 = b4.nodes.size();
    std::vector<Node4> nodes(8 * n4);
    for (int oct = 0; oct < 8; ++oct)
        for (size_t k = 0; k < n4; ++k) {
            const auto& s = b4.nodes[k];
            Node4& d = nodes[oct * n4 + k];
            float* nr[3] = {d.nx, d.ny, d.nz};
            float* fr[3] = {d.fx, d.fy, d.fz};
            for (uint32_t q = 0; q < 4; ++q) {
                const uint32_t slot = s.order[oct][q];
                const bool valid = q < s.n;
                for (int a = 0; a < 3; ++a) {
                    const bool neg = (oct >> a) & 1;
                    const float lo = valid ? down(s.lo[slot][a]) : INFINITY;
                    const float hi = valid ? up(s.hi[slot][a]) : -INFINITY;
                    nr[a][q] = neg ? hi : lo;
                    fr[a][q] = neg ? lo : hi;
                }
                d.child[q] = valid ? s.child[slot] : rtw::leaf_code(0, 0);
            }
        }
    // traversal restated (render_kernel.hpp bvh4_traverse, one lane)
    std::uniform_real_distribution<double> D(-1, 1), O(-14, 14);
    long visits = 0, tests = 0;
    int max_sp = 0;
    const int rays = 200000;
    for (int r = 0; r < rays; ++r) {
        float o[3] = {(float)O(g), (float)(D(g) * 3 + 2), (float)O(g)};
        float d[3] = {(float)D(g), (float)D(g), (float)D(g)};
        if (r % 50 == 0) d[r / 50 % 3] = (r & 64) ? -0.0f : 0.0f;   // axis-parallel rays
        const float ix = 1.f / d[0], iy = 1.f / d[1], iz = 1.f / d[2];
        const float oix = o[0] * ix, oiy = o[1] * iy, oiz = o[2] * iz;
        const uint32_t oct = (signbit(ix) ? 1 : 0) | (signbit(iy) ? 2 : 0) | (signbit(iz) ? 4 : 0);
        const Node4* base = nodes.data() + oct * n4;
        // brute force, f64 (exact reference is not the point: closest id)
        auto hit_t = [&](uint32_t k, double& t) {
            const double* s = &sph[4 * k];
            const double ocx = o[0] - s[0], ocy = o[1] - s[1], ocz = o[2] - s[2];
            const double a = (double)d[0] * d[0] + (double)d[1] * d[1] + (double)d[2] * d[2];
            const double hb = ocx * d[0] + ocy * d[1] + ocz * d[2];
            const double c = ocx * ocx + ocy * ocy + ocz * ocz - s[3] * s[3];
            const double disc = hb * hb - a * c;
            if (disc < 0) return false;
            const double sq = sqrt(disc);
            t = (-hb - sq) / a;
            if (t < 1e-4) t = (-hb + sq) / a;
            return t >= 1e-4;
        };
        double tb_ref = INFINITY;
        int best_ref = -1;
        for (uint32_t k = 0; k < n; ++k) {
            double t;
            if (hit_t(k, t) && t < tb_ref) tb_ref = t, best_ref = (int)k;
        }
        int32_t stk[64];
        int sp = 0;
        int32_t node = 0;
        double tb = INFINITY;
        int best = -1;
        for (;;) {
            if (node >= 0) {
                ++visits;
                const Node4& nd = base[node];
                bool h[4];
                const float tbf = (float)tb;
                for (int c = 0; c < 4; ++c) {
                    const float xn = fmaf(nd.nx[c], ix, -oix), xf = fmaf(nd.fx[c], ix, -oix);
                    const float yn = fmaf(nd.ny[c], iy, -oiy), yf = fmaf(nd.fy[c], iy, -oiy);
                    const float zn = fmaf(nd.nz[c], iz, -oiz), zf = fmaf(nd.fz[c], iz, -oiz);
                    const float tn = fmaxf(fmaxf(xn, yn), fmaxf(zn, 0.f));
                    const float tf = fminf(fminf(xf, yf), fminf(zf, tbf));
                    h[c] = tn <= tf;
                }
                stk[sp] = nd.child[3];
                sp += (h[3] && (h[0] || h[1] || h[2]));
                stk[sp] = nd.child[2];
                sp += (h[2] && (h[0] || h[1]));
                stk[sp] = nd.child[1];
                sp += (h[1] && h[0]);
                max_sp = std::max(max_sp, sp);
                if (h[0] | h[1] | h[2] | h[3])
                    node = h[0] ? nd.child[0] : (h[1] ? nd.child[1] : (h[2] ? nd.child[2] : nd.child[3]));
                else if (sp)
                    node = stk[--sp];
                else
                    break;
            } else {
                const uint32_t code = ~(uint32_t)node;
                for (uint32_t k = 0; k < (code & 15u); ++k) {
                    const uint32_t id = bb.order[(code >> 4) + k];
                    double t;
                    ++tests;
                    if (hit_t(id, t) && (t < tb || (t == tb && (int)id < best))) tb = t, best = (int)id;
                }
                if (!sp) break;
                node = stk[--sp];
            }
        }
        CHECK(best == best_ref, "ray %d: bvh4 %d vs brute %d (t %.9g vs %.9g)", r, best, best_ref, tb, tb_ref);
        if (fails > 10) return 1;
    }
    CHECK(max_sp <= (int)b4.max_stack, "stack %d > bound %u", max_sp, b4.max_stack);
    printf("rays %d: %.2f node visits, %.2f sphere tests per ray, max stack %d (bound %u)\n", rays,
           (double)visits / rays, (double)tests / rays, max_sp, b4.max_stack);
    printf(fails ? "FAILED\n" : "OK\n");
    return fails ? 1 : 0;
}
