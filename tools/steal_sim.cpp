// steal_sim.cpp -- lockstep simulation of the kernel's while-while BVH
// traversal (render_kernel.hpp bvh_traverse_ww) over the ray batches of
// tools/steal_sim.py, with and without intra-wave subtree stealing: a lane
// with nothing left to traverse (its own ray done, or skipped) takes the
// bottom entry of another lane's stack together with that lane's ray, and
// the partial results are folded into the owner's (t, id) minimum.
// Counts inner-node passes, leaf passes, steal rounds and lanes per pass,
// and checks every lane's closest hit against brute force.
//   g++ -O2 -std=c++17 -I ray_tracing_weekend_amd/csrc tools/steal_sim.cpp \
//       ray_tracing_weekend_amd/csrc/host/bvh.cpp -o /tmp/steal_sim && /tmp/steal_sim rays.bin
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#include "host/bvh.hpp"

constexpr int kLanes = 64;
constexpr int32_t kDone = 0x7fffffff;

struct Ray {
    double o[3], d[3];
    int32_t excl, skip, active;
};

struct Res {
    double t = INFINITY;
    int32_t id = -1;
    bool better(double t2, int32_t id2) const { return t2 < t || (t2 == t && (uint32_t)id2 < (uint32_t)id); }
};

int main(int argc, char** argv) {
    if (argc < 2) return 2;
    FILE* f = fopen(argv[1], "rb");
    if (!f) return 2;
    uint32_t n_sph = 0, n_b = 0;
    if (fread(&n_sph, 4, 1, f) != 1 || fread(&n_b, 4, 1, f) != 1) return 2;
    std::vector<double> sph(4 * n_sph);
    if (fread(sph.data(), 8, sph.size(), f) != sph.size()) return 2;
    std::vector<Ray> rays((size_t)n_b * kLanes);
    for (auto& r : rays)
        if (fread(r.o, 8, 3, f) != 3 || fread(r.d, 8, 3, f) != 3 || fread(&r.excl, 4, 1, f) != 1 ||
            fread(&r.skip, 4, 1, f) != 1 || fread(&r.active, 4, 1, f) != 1)
            return 2;
    fclose(f);
    const rtw::BvhBuild bb = rtw::build_bvh(sph.data(), n_sph, 1e-5, 4);
    auto hit_t = [&](uint32_t k, const double* o, const double* d, double& t) {
        const double* s = &sph[4 * k];
        const double oc[3] = {o[0] - s[0], o[1] - s[1], o[2] - s[2]};
        const double a = d[0] * d[0] + d[1] * d[1] + d[2] * d[2];
        const double hb = oc[0] * d[0] + oc[1] * d[1] + oc[2] * d[2];
        const double c = oc[0] * oc[0] + oc[1] * oc[1] + oc[2] * oc[2] - s[3] * s[3];
        const double disc = hb * hb - a * c;
        if (!(disc > 0)) return false;
        const double eps = 2.220446049250313e-16;
        t = (-hb - sqrt(disc)) / a;
        if (!(t >= eps)) t = (-hb + sqrt(disc)) / a;
        return t >= eps;
    };
    const int mode_lo = argc > 2 ? atoi(argv[2]) : 0, mode_hi = argc > 3 ? atoi(argv[3]) : 2;
    for (int mode = mode_lo; mode <= mode_hi; ++mode) {
        // mode 0: the kernel; 1: + stealing the bottom stack entry; 2: + the
        // bound shared through the owner's key at every leaf phase and steal;
        // 3: as 2, stealing the top entry instead
        long inner_passes = 0, inner_lanes = 0, leaf_passes = 0, leaf_lanes = 0, steal_rounds = 0, steals = 0;
        long visits = 0, fails = 0, segs = 0, checks = 0;
        for (uint32_t b = 0; b < n_b; ++b) {
            const Ray* R = &rays[(size_t)b * kLanes];
            struct Lane {
                int32_t owner = -1;      // ray being traversed (lane index), -1 none
                int32_t node = kDone, leaf = 0, sp = 0, base = 0;
                int32_t stk[64];
                Res r;                   // running result of the current context
                bool act = false;
            } L[kLanes];
            Res slot[kLanes];
            for (int k = 0; k < kLanes; ++k) {
                L[k].act = R[k].active != 0;
                if (!L[k].act) continue;
                ++segs;
                L[k].owner = k;
                L[k].node = R[k].skip ? kDone : 0;
                if (R[k].skip) {         // own isolated sphere re-hit: its t is the answer
                    double t = INFINITY;
                    hit_t((uint32_t)R[k].excl, R[k].o, R[k].d, t);
                    slot[k] = Res{t, R[k].excl};
                }
            }
            auto fold = [&](Lane& l) {   // a finished context: into the owner's slot
                if (l.owner >= 0 && slot[l.owner].better(l.r.t, l.r.id)) slot[l.owner] = l.r;
                l.r = Res{};
                l.owner = -1;
            };
            auto step = [&](Lane& l) {
                const Ray& ray = R[l.owner];
                const auto& nd = bb.nodes[l.node];
                double tn[2], tf[2];
                for (int c = 0; c < 2; ++c) {
                    double lo = 0, hi = INFINITY;
                    for (int a = 0; a < 3; ++a) {
                        const double ix = 1.0 / ray.d[a];
                        double t0 = (nd.lo[c][a] - ray.o[a]) * ix, t1 = (nd.hi[c][a] - ray.o[a]) * ix;
                        if (t0 != t0) t0 = -INFINITY;
                        if (t1 != t1) t1 = INFINITY;
                        lo = std::max(lo, std::min(t0, t1));
                        hi = std::min(hi, std::max(t0, t1));
                    }
                    tn[c] = lo;
                    tf[c] = std::min(hi, l.r.t);
                }
                const bool h0 = tn[0] <= tf[0], h1 = tn[1] <= tf[1];
                const int32_t c0 = nd.child[0], c1 = nd.child[1];
                if (h0 && h1) {
                    const bool first0 = tn[0] <= tn[1];
                    l.stk[l.sp++] = first0 ? c1 : c0;
                    l.node = first0 ? c0 : c1;
                } else if (h0 || h1) {
                    l.node = h0 ? c0 : c1;
                } else {
                    l.node = l.sp > l.base ? l.stk[--l.sp] : kDone;
                }
                ++visits;
            };
            auto test_leaf = [&](Lane& l) {
                const Ray& ray = R[l.owner];
                const uint32_t code = ~(uint32_t)l.leaf;
                for (uint32_t k = 0; k < (code & 15u); ++k) {
                    const uint32_t id = bb.order[(code >> 4) + k];
                    double t;
                    if ((int32_t)id != ray.excl && hit_t(id, ray.o, ray.d, t) && l.r.better(t, (int32_t)id))
                        l.r = Res{t, (int32_t)id};
                }
                l.leaf = 0;
            };
            // steal round: idle lanes (k-th) take the bottom stack entry of donors (k-th)
            auto steal = [&]() {
                int idle[kLanes], donor[kLanes], ni = 0, nd = 0;
                for (int k = 0; k < kLanes; ++k) {
                    Lane& l = L[k];
                    if (!l.act) continue;
                    if (l.node == kDone && l.leaf == 0) idle[ni++] = k;
                    else if (l.sp > l.base) donor[nd++] = k;
                }
                const int np = std::min(ni, nd);
                if (np == 0) return false;
                ++steal_rounds;
                for (int q = 0; q < np; ++q) {
                    Lane& t = L[idle[q]];
                    Lane& d = L[donor[q]];
                    fold(t);
                    t.owner = d.owner;
                    t.r = d.r;
                    if (mode >= 2 && slot[t.owner].better(t.r.t, t.r.id) == false) t.r = slot[t.owner];
                    t.node = mode == 3 ? d.stk[--d.sp] : d.stk[d.base++];
                    t.sp = t.base = 0;
                    ++steals;
                }
                return true;
            };
            for (int guard = 0;; ++guard) {
                if (guard > 100000) {
                    printf("FAIL: no termination\n");
                    return 1;
                }
                for (int it = 0;; ++it) {
                    bool any_inner = false, all_wait = true;
                    for (auto& l : L) {
                        if (!l.act) continue;
                        if (l.node < 0 && l.leaf == 0) {
                            l.leaf = l.node;
                            l.node = l.sp > l.base ? l.stk[--l.sp] : kDone;
                        }
                        if (mode && l.node == kDone && l.leaf == 0) fold(l);
                    }
                    if (mode) steal();
                    for (auto& l : L) {
                        if (!l.act) continue;
                        if (l.node < 0 && l.leaf == 0) {
                            l.leaf = l.node;
                            l.node = l.sp > l.base ? l.stk[--l.sp] : kDone;
                        }
                        const bool inner = l.node >= 0 && l.node != kDone;
                        any_inner |= inner;
                        all_wait &= l.leaf != 0 || l.node == kDone;
                    }
                    if (!any_inner || all_wait) break;
                    ++inner_passes;
                    for (auto& l : L)
                        if (l.act && l.node >= 0 && l.node != kDone) {
                            ++inner_lanes;
                            step(l);
                        }
                }
                bool any_leaf = false;
                for (auto& l : L) any_leaf |= l.act && l.leaf != 0;
                if (!any_leaf) {
                    // mode 1/2: a stealable entry may still be left (a lane
                    // holding stack entries always has inner work, so no)
                    break;
                }
                ++leaf_passes;
                for (auto& l : L)
                    if (l.act && l.leaf != 0) {
                        ++leaf_lanes;
                        test_leaf(l);
                        if (mode >= 2) {   // share the bound through the owner's key
                            if (slot[l.owner].better(l.r.t, l.r.id)) slot[l.owner] = l.r;
                            else l.r = slot[l.owner];
                        }
                    }
            }
            for (auto& l : L)
                if (l.act) fold(l);
            for (int k = 0; k < kLanes; ++k) {
                if (!L[k].act) continue;
                if (L[k].node != kDone || L[k].sp != L[k].base) {
                    printf("FAIL: lane %d not finished\n", k);
                    return 1;
                }
                // brute force
                Res bf;
                for (uint32_t s = 0; s < n_sph; ++s) {
                    double t;
                    if ((int32_t)s != R[k].excl && hit_t(s, R[k].o, R[k].d, t) && bf.better(t, (int32_t)s))
                        bf = Res{t, (int32_t)s};
                }
                if (R[k].skip) {
                    double t = INFINITY;
                    hit_t((uint32_t)R[k].excl, R[k].o, R[k].d, t);
                    if (bf.better(t, R[k].excl) || true) bf = Res{t, R[k].excl};   // provably closest
                }
                ++checks;
                if (bf.id != slot[k].id && ++fails < 5)
                    printf("FAIL batch %u lane %d: %d vs brute %d\n", b, k, slot[k].id, bf.id);
            }
        }
        const double per64 = 64.0 / segs;
        printf("mode %d: inner passes %.2f (lanes %.1f), leaf passes %.2f (lanes %.1f), steal rounds %.2f (%.1f "
               "steals) per 64 segments; visits/seg %.2f; fails %ld of %ld\n",
               mode, inner_passes * per64, (double)inner_lanes / std::max(inner_passes, 1L), leaf_passes * per64,
               (double)leaf_lanes / std::max(leaf_passes, 1L), steal_rounds * per64,
               (double)steals / std::max(steal_rounds, 1L), visits / (double)segs, fails, checks);
        printf("        cost 46/inner + 118/leaf + 30/steal round + 8/inner (mode>0 check) = %.0f VALU per 64 segments\n",
               (46.0 * inner_passes + 118.0 * leaf_passes + 30.0 * steal_rounds + (mode ? 8.0 * inner_passes : 0)) *
                   per64);
    }
    return 0;
}
