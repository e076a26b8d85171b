// ww_check.cpp -- host-only lockstep simulation of the binary while-while
// traversal in render_kernel.hpp (bvh_traverse_ww): 64 lanes execute the
// same iteration with the kernel's wave-uniform loop conditions; every lane's
// closest sphere must equal brute force, every wave must terminate, and the
// stack must stay within `depth` entries (the kernel sizes it so).
//   g++ -O2 -std=c++17 -I ray_tracing_weekend_amd/csrc tools/ww_check.cpp \
//       ray_tracing_weekend_amd/csrc/host/bvh.cpp -o /tmp/ww_check && /tmp/ww_check
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <random>
#include <vector>

#include "host/bvh.hpp"

constexpr int kLanes = 64;
constexpr int32_t kDone = 0x7fffffff;

int main(int argc, char** argv) {
    const uint32_t n = argc > 1 ? (uint32_t)atoi(argv[1]) : 484;
    // leaf phase once every lane holds a leaf or is done (the kernel), or once
    // `thr` lanes hold one
    const int thr = argc > 2 ? atoi(argv[2]) : 64;
    long leaf_phases = 0;
    std::mt19937_64 g(3);
    std::uniform_real_distribution<double> U(-11, 11), Rr(0.05, 0.3), D(-1, 1), O(-14, 14);
    std::vector<double> sph(4 * n);
    for (uint32_t k = 0; k < n; ++k) {
        sph[4 * k] = U(g);
        sph[4 * k + 1] = k % 7 == 0 ? 1.0 : 0.2;
        sph[4 * k + 2] = U(g);
        sph[4 * k + 3] = k % 7 == 0 ? 1.0 : Rr(g);
    }
    const rtw::BvhBuild bb = rtw::build_bvh(sph.data(), n, 1e-5);
    const int cap = (int)bb.depth;
    auto hit_t = [&](uint32_t k, const double* o, const double* d, double& t) {
        const double* s = &sph[4 * k];
        const double oc[3] = {o[0] - s[0], o[1] - s[1], o[2] - s[2]};
        const double a = d[0] * d[0] + d[1] * d[1] + d[2] * d[2];
        const double hb = oc[0] * d[0] + oc[1] * d[1] + oc[2] * d[2];
        const double c = oc[0] * oc[0] + oc[1] * oc[1] + oc[2] * oc[2] - s[3] * s[3];
        const double disc = hb * hb - a * c;
        if (disc < 0) return false;
        t = (-hb - sqrt(disc)) / a;
        if (t < 1e-4) t = (-hb + sqrt(disc)) / a;
        return t >= 1e-4;
    };
    long fails = 0, iters = 0, visits = 0;
    int max_sp = 0;
    for (int wave = 0; wave < 3000; ++wave) {
        struct Lane {
            double o[3], d[3], ix[3];
            int32_t sp = 0, top = kDone, node = 0, leaf = 0;
            double tb = INFINITY;
            int best = -1;
            int32_t stk[64];
        } L[kLanes];
        for (auto& l : L) {
            for (int a = 0; a < 3; ++a) {
                l.o[a] = a == 1 ? D(g) * 3 + 2 : O(g);
                l.d[a] = D(g);
            }
            if (wave % 5 == 0) l.d[wave % 3] = 0.0;
            for (int a = 0; a < 3; ++a) l.ix[a] = 1.0 / l.d[a];
            for (auto& e : l.stk) e = 12345678;   // junk
        }
        long guard = 0;
        for (;;) {
            for (;;) {
                bool any_busy = false, all_wait = true;
                int holding = 0;
                for (auto& l : L) {
                    const bool park = l.node < 0 && l.leaf == 0;
                    any_busy |= park || (l.node >= 0 && l.node != kDone);
                    all_wait &= l.leaf != 0 || l.node == kDone;
                    holding += l.leaf != 0;
                }
                if (!any_busy || all_wait || holding >= thr) break;
                if (++guard > 100000) {
                    printf("FAIL: wave %d does not terminate\n", wave);
                    return 1;
                }
                ++iters;
                for (auto& l : L) {
                    int32_t& sp = l.sp;
                    const bool park = l.node < 0 && l.leaf == 0;
                    l.leaf = park ? l.node : l.leaf;
                    const int32_t cur = park ? (sp > 0 ? l.top : kDone) : l.node;
                    sp -= (park && sp > 0) ? 1 : 0;
                    const int32_t refill1 = l.stk[sp > 0 ? sp - 1 : 0];
                    const bool inner = cur >= 0 && cur != kDone;
                    const auto& nd = bb.nodes[inner ? cur : 0];
                    double tn[2], tf[2];
                    for (int c = 0; c < 2; ++c) {
                        double lo = 0, hi = INFINITY;
                        for (int a = 0; a < 3; ++a) {
                            double t0 = (nd.lo[c][a] - l.o[a]) * l.ix[a], t1 = (nd.hi[c][a] - l.o[a]) * l.ix[a];
                            if (t0 != t0) t0 = -INFINITY;
                            if (t1 != t1) t1 = INFINITY;
                            lo = std::max(lo, std::min(t0, t1));
                            hi = std::min(hi, std::max(t0, t1));
                        }
                        tn[c] = lo;
                        tf[c] = std::min(hi, l.tb);
                    }
                    l.top = park ? refill1 : l.top;
                    const bool h0 = inner && tn[0] <= tf[0], h1 = inner && tn[1] <= tf[1];
                    const int32_t c0 = nd.child[0], c1 = nd.child[1];
                    const bool both = h0 && h1, any = h0 || h1;
                    const bool first0 = tn[0] <= tn[1];
                    const int32_t farc = first0 ? c1 : c0;
                    const int32_t child = both ? (first0 ? c0 : c1) : (h0 ? c0 : c1);
                    const bool pop = inner && !any;
                    if (sp >= cap) {
                        printf("FAIL: stack store at %d >= %d\n", sp, cap);
                        return 1;
                    }
                    l.stk[sp] = farc;
                    const int32_t next = inner ? (any ? child : (sp > 0 ? l.top : kDone)) : cur;
                    sp -= (pop && sp > 0) ? 1 : 0;
                    const int32_t refill2 = l.stk[sp > 0 ? sp - 1 : 0];
                    l.top = both ? farc : (pop ? refill2 : l.top);
                    sp += both ? 1 : 0;
                    max_sp = std::max(max_sp, (int)sp);
                    l.node = next;
                    visits += inner;
                }
            }
            bool any_leaf = false, all_done = true;
            for (auto& l : L) {
                any_leaf |= l.leaf != 0;
                all_done &= l.node == kDone && l.leaf == 0;
            }
            if (all_done) break;
            if (!any_leaf) continue;
            ++leaf_phases;
            for (auto& l : L) {
                if (l.leaf == 0) continue;
                const uint32_t code = ~(uint32_t)l.leaf;
                for (uint32_t k = 0; k < (code & 15u); ++k) {
                    const uint32_t id = bb.order[(code >> 4) + k];
                    double t;
                    if (hit_t(id, l.o, l.d, t) && (t < l.tb || (t == l.tb && (int)id < l.best))) {
                        l.tb = t;
                        l.best = (int)id;
                    }
                }
                l.leaf = 0;
            }
        }
        for (auto& l : L) {
            if (l.node != kDone || l.sp != 0) {
                printf("FAIL: lane not finished (node %d sp %d)\n", l.node, l.sp);
                return 1;
            }
            double tb = INFINITY;
            int best = -1;
            for (uint32_t k = 0; k < n; ++k) {
                double t;
                if (hit_t(k, l.o, l.d, t) && t < tb) tb = t, best = (int)k;
            }
            if (best != l.best && ++fails < 10) printf("FAIL: best %d vs brute %d\n", l.best, best);
        }
    }
    printf("thr %d: leaf phases %ld, cost model 50*iters + 110*leaf = %.0f per wave\n", thr, leaf_phases,
           (50.0 * iters + 110.0 * leaf_phases) / 3000);
    printf("n=%u depth=%u: %ld wave iterations, %.2f visits/ray, max stack %d (cap %d), fails %ld\n", n,
           bb.depth, iters, visits / (3000.0 * kLanes), max_sp, cap, fails);
    printf(fails ? "FAILED\n" : "OK\n");
    return fails ? 1 : 0;
}
