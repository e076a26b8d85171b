// bvh.cpp -- binned-SAH BVH build over spheres (see bvh.hpp).
#include "bvh.hpp"

#include <string.h>


#include <math.h>

#include <cmath>
#include <algorithm>
#include <numeric>

namespace rtw {
namespace {

struct Box {
    double lo[3] = {INFINITY, INFINITY, INFINITY};
    double hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    void grow(const Box& b) {
        for (int k = 0; k < 3; ++k) {
            lo[k] = std::min(lo[k], b.lo[k]);
            hi[k] = std::max(hi[k], b.hi[k]);
        }
    }
    void grow_pt(const double* p) {
        for (int k = 0; k < 3; ++k) {
            lo[k] = std::min(lo[k], p[k]);
            hi[k] = std::max(hi[k], p[k]);
        }
    }
    double area() const {
        double dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
        if (!(dx >= 0) || !(dy >= 0) || !(dz >= 0)) return 0.0;
        return 2.0 * (dx * dy + dx * dz + dy * dz);
    }
};

struct Prim {
    Box box;
    double c[3];
    uint32_t id;
};

struct Builder {
    std::vector<Prim> prims;
    BvhBuild* out;
    double pad;
    uint32_t leaf_max;

    Box padded(Box b) const {
        for (int k = 0; k < 3; ++k) {
            b.lo[k] -= pad;
            b.hi[k] += pad;
        }
        return b;
    }

    // returns the child code for prims [b, e) and fills its box
    int32_t build(uint32_t b, uint32_t e, uint32_t level, Box* box_out) {
        Box box;
        for (uint32_t k = b; k < e; ++k) box.grow(prims[k].box);
        *box_out = padded(box);
        const uint32_t n = e - b;
        if (n <= leaf_max) {
            std::sort(prims.begin() + b, prims.begin() + e,
                      [](const Prim& x, const Prim& y) { return x.id < y.id; });
            const uint32_t first = (uint32_t)out->order.size();
            for (uint32_t k = b; k < e; ++k) out->order.push_back(prims[k].id);
            out->leaves++;
            out->depth = std::max(out->depth, level);
            return leaf_code(first, n);
        }
        Box cb;
        for (uint32_t k = b; k < e; ++k) cb.grow_pt(prims[k].c);
        constexpr int kBins = 16;
        double best_cost = INFINITY;
        int best_axis = -1, best_split = 0;
        for (int axis = 0; axis < 3; ++axis) {
            const double ext = cb.hi[axis] - cb.lo[axis];
            if (!(ext > 0)) continue;
            Box bins[kBins];
            uint32_t cnt[kBins] = {};
            const double scale = kBins / ext;
            for (uint32_t k = b; k < e; ++k) {
                int bi = std::min(kBins - 1, (int)((prims[k].c[axis] - cb.lo[axis]) * scale));
                cnt[bi]++;
                bins[bi].grow(prims[k].box);
            }
            double right_area[kBins];
            uint32_t right_cnt[kBins];
            Box acc;
            uint32_t c = 0;
            for (int s = kBins - 1; s > 0; --s) {
                acc.grow(bins[s]);
                c += cnt[s];
                right_area[s] = acc.area();
                right_cnt[s] = c;
            }
            Box lacc;
            uint32_t lc = 0;
            for (int s = 1; s < kBins; ++s) {
                lacc.grow(bins[s - 1]);
                lc += cnt[s - 1];
                if (lc == 0 || right_cnt[s] == 0) continue;
                const double cost = lacc.area() * lc + right_area[s] * right_cnt[s];
                if (cost < best_cost) {
                    best_cost = cost;
                    best_axis = axis;
                    best_split = s;
                }
            }
        }
        uint32_t mid;
        if (best_axis < 0) {
            mid = b + n / 2;   // coincident centroids: split by index
        } else {
            const double ext = cb.hi[best_axis] - cb.lo[best_axis];
            const double scale = kBins / ext;
            auto it = std::partition(prims.begin() + b, prims.begin() + e, [&](const Prim& p) {
                int bi = std::min(kBins - 1, (int)((p.c[best_axis] - cb.lo[best_axis]) * scale));
                return bi < best_split;
            });
            mid = (uint32_t)(it - prims.begin());
            if (mid == b || mid == e) mid = b + n / 2;
        }
        const int32_t node = (int32_t)out->nodes.size();
        out->nodes.emplace_back();
        Box lb, rb;
        const int32_t l = build(b, mid, level + 1, &lb);
        const int32_t r = build(mid, e, level + 1, &rb);
        BvhBuild::Node& nd = out->nodes[node];
        for (int k = 0; k < 3; ++k) {
            nd.lo[0][k] = lb.lo[k];
            nd.hi[0][k] = lb.hi[k];
            nd.lo[1][k] = rb.lo[k];
            nd.hi[1][k] = rb.hi[k];
        }
        nd.child[0] = l;
        nd.child[1] = r;
        return node;
    }
};

}  // namespace

BvhBuild build_bvh(const double* spheres, uint32_t n, double pad_rel, uint32_t leaf_max) {
    BvhBuild out;
    Builder bld;
    bld.out = &out;
    bld.leaf_max = leaf_max < 1 ? 1 : (leaf_max > 15 ? 15 : leaf_max);
    bld.prims.resize(n);
    double scale = 0.0;
    for (uint32_t k = 0; k < n; ++k) {
        const double* s = spheres + 4 * k;
        Prim& p = bld.prims[k];
        const double r = fabs(s[3]);
        for (int a = 0; a < 3; ++a) {
            p.box.lo[a] = s[a] - r;
            p.box.hi[a] = s[a] + r;
            p.c[a] = s[a];
            scale = std::max(scale, fabs(s[a]) + r);
        }
        p.id = k;
    }
    bld.pad = pad_rel * (scale + 1.0);
    out.order.reserve(n);
    out.nodes.reserve(n ? 2 * (n / bld.leaf_max + 1) : 1);
    // the root is always an inner node (an empty right child when n <= leaf_max)
    if (n <= bld.leaf_max) {
        out.nodes.emplace_back();
        Box lb;
        int32_t l = n ? bld.build(0, n, 1, &lb) : leaf_code(0, 0);
        BvhBuild::Node& nd = out.nodes[0];
        for (int k = 0; k < 3; ++k) {
            nd.lo[0][k] = n ? lb.lo[k] : INFINITY;
            nd.hi[0][k] = n ? lb.hi[k] : -INFINITY;
            nd.lo[1][k] = INFINITY;
            nd.hi[1][k] = -INFINITY;
        }
        nd.child[0] = l;
        nd.child[1] = leaf_code(0, 0);
        out.depth = 1;
    } else {
        Box root;
        bld.build(0, n, 0, &root);
    }
    return out;
}

namespace {

struct Collapser {
    const BvhBuild& b;
    Bvh4Build& out;

    static double area(const double* lo, const double* hi) {
        const double dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
        if (!(dx >= 0) || !(dy >= 0) || !(dz >= 0)) return 0.0;
        return dx * dy + dx * dz + dy * dz;
    }

    // a child slot: child `side` of binary node `parent`
    struct Ref {
        int32_t parent;
        int side;
    };

    // front-to-back order (slot indices) of the final children below binary
    // node `node` for octant `oct` (bit a set: the ray goes -a); `opened`
    // holds the binary nodes that were opened into this 4-wide node
    void order(int32_t node, const std::vector<int32_t>& opened, const std::vector<Ref>& slots, int oct,
               std::vector<int>& seq) const {
        const BvhBuild::Node& nd = b.nodes[node];
        // split axis: the largest separation of the two child box centres
        int axis = 0;
        double best = -1.0;
        for (int a = 0; a < 3; ++a) {
            const double c0 = nd.lo[0][a] + nd.hi[0][a], c1 = nd.lo[1][a] + nd.hi[1][a];
            const double sep = fabs(c1 - c0);
            if (std::isfinite(sep) && sep > best) {
                best = sep;
                axis = a;
            }
        }
        const double c0 = nd.lo[0][axis] + nd.hi[0][axis], c1 = nd.lo[1][axis] + nd.hi[1][axis];
        const bool neg = (oct >> axis) & 1;
        int first = (c0 <= c1) ? 0 : 1;
        if (neg) first ^= 1;
        for (int side : {first, first ^ 1}) {
            const int32_t ch = nd.child[side];
            if (ch >= 0 && std::find(opened.begin(), opened.end(), ch) != opened.end()) {
                order(ch, opened, slots, oct, seq);
            } else {
                for (size_t k = 0; k < slots.size(); ++k)
                    if (slots[k].parent == node && slots[k].side == side) seq.push_back((int)k);
            }
        }
    }

    // emit the 4-wide node rooted at binary inner node `bn`; returns its index
    int32_t emit(int32_t bn, uint32_t level, uint32_t* stack_need) {
        std::vector<Ref> slots = {{bn, 0}, {bn, 1}};
        std::vector<int32_t> opened = {bn};
        while (slots.size() < 4) {
            int pick = -1;
            double best = -1.0;
            for (size_t k = 0; k < slots.size(); ++k) {
                const int32_t ch = b.nodes[slots[k].parent].child[slots[k].side];
                if (ch < 0) continue;
                const BvhBuild::Node& p = b.nodes[slots[k].parent];
                const double a = area(p.lo[slots[k].side], p.hi[slots[k].side]);
                if (a > best) {
                    best = a;
                    pick = (int)k;
                }
            }
            if (pick < 0) break;
            const int32_t ch = b.nodes[slots[pick].parent].child[slots[pick].side];
            slots.erase(slots.begin() + pick);
            slots.push_back({ch, 0});
            slots.push_back({ch, 1});
            opened.push_back(ch);
        }
        // drop empty leaves (the root's padding child of a tiny scene)
        slots.erase(std::remove_if(slots.begin(), slots.end(),
                                   [&](const Ref& r) {
                                       const int32_t ch = b.nodes[r.parent].child[r.side];
                                       return ch < 0 && (((uint32_t)~ch) & 15u) == 0;
                                   }),
                    slots.end());
        const int32_t idx = (int32_t)out.nodes.size();
        out.nodes.emplace_back();
        out.depth = std::max(out.depth, level + 1);
        Bvh4Build::Node nd{};
        nd.n = (uint32_t)slots.size();
        for (int k = 0; k < 4; ++k) {
            nd.child[k] = leaf_code(0, 0);
            for (int a = 0; a < 3; ++a) {
                nd.lo[k][a] = INFINITY;
                nd.hi[k][a] = -INFINITY;
            }
        }
        for (int oct = 0; oct < 8; ++oct) {
            std::vector<int> seq;
            order(bn, opened, slots, oct, seq);
            for (int k = 0; k < 4; ++k) nd.order[oct][k] = (uint8_t)(k < (int)seq.size() ? seq[k] : k);
        }
        uint32_t below = 0;
        for (size_t k = 0; k < slots.size(); ++k) {
            const BvhBuild::Node& p = b.nodes[slots[k].parent];
            for (int a = 0; a < 3; ++a) {
                nd.lo[k][a] = p.lo[slots[k].side][a];
                nd.hi[k][a] = p.hi[slots[k].side][a];
            }
            const int32_t ch = p.child[slots[k].side];
            if (ch >= 0) {
                uint32_t need = 0;
                nd.child[k] = emit(ch, level + 1, &need);
                below = std::max(below, need);
            } else {
                nd.child[k] = ch;
            }
        }
        out.nodes[idx] = nd;
        *stack_need = (nd.n ? nd.n - 1 : 0) + below;
        return idx;
    }
};

}  // namespace

std::vector<uint8_t> isolated_spheres(const double* spheres, uint32_t n, const BvhBuild& b, double margin) {
    std::vector<uint8_t> iso(n, 0);
    if (b.nodes.empty()) return iso;
    std::vector<int32_t> stack;
    for (uint32_t i = 0; i < n; ++i) {
        const double* si = spheres + 4 * i;
        if (!(si[3] >= 0)) continue;
        const double reach = si[3] + margin;
        double lo[3], hi[3];
        for (int a = 0; a < 3; ++a) {
            lo[a] = si[a] - reach;
            hi[a] = si[a] + reach;
        }
        bool alone = true;
        stack.clear();
        stack.push_back(0);
        while (alone && !stack.empty()) {
            const int32_t node = stack.back();
            stack.pop_back();
            if (node >= 0) {
                const BvhBuild::Node& nd = b.nodes[node];
                for (int c = 0; c < 2; ++c) {
                    bool overlap = true;
                    for (int a = 0; a < 3; ++a)
                        overlap = overlap && nd.lo[c][a] <= hi[a] && nd.hi[c][a] >= lo[a];
                    if (overlap) stack.push_back(nd.child[c]);
                }
            } else {
                const uint32_t code = ~(uint32_t)node;
                for (uint32_t k = 0; k < (code & 15u) && alone; ++k) {
                    const uint32_t j = b.order[(code >> 4) + k];
                    if (j == i) continue;
                    const double* sj = spheres + 4 * j;
                    if (!(sj[3] >= 0)) continue;
                    const double dx = si[0] - sj[0], dy = si[1] - sj[1], dz = si[2] - sj[2];
                    const double lim = si[3] + sj[3] + margin;
                    if (dx * dx + dy * dy + dz * dz <= lim * lim) alone = false;
                }
            }
        }
        iso[i] = alone ? 1 : 0;
    }
    return iso;
}

Bvh4Build collapse_bvh4(const BvhBuild& b) {
    Bvh4Build out;
    if (b.nodes.empty()) return out;
    Collapser c{b, out};
    uint32_t need = 0;
    c.emit(0, 0, &need);
    out.max_stack = need;
    return out;
}

LightGrid build_light_grid(const double* L, uint32_t n, double cells_per_light) {
    LightGrid g;
    std::vector<uint8_t> big(n, 0);
    for (uint32_t k = 0; k < n; ++k)
        for (int a = 0; a < 4; ++a)
            if (!std::isfinite(L[4 * k + a])) big[k] = 1;
    // lights much larger than the typical one would stretch the grid box (the
    // scenes::simple field: r = 0.2 lights at y = 0.2 and one r = 1 sphere --
    // with it the box is 5x as tall and grazing rays walk 5x as far)
    {
        std::vector<double> r;
        for (uint32_t k = 0; k < n; ++k)
            if (!big[k]) r.push_back(fabs(L[4 * k + 3]));
        if (!r.empty()) {
            std::nth_element(r.begin(), r.begin() + r.size() / 2, r.end());
            const double med = r[r.size() / 2];
            for (uint32_t k = 0; k < n; ++k)
                if (!big[k] && fabs(L[4 * k + 3]) > kGridBigRadius * med) big[k] = 1;
        }
    }
    // cells overlapped by light k's AABB, padded by more than the rounding of
    // the kernel's cell walk and closest-approach parameter (f32 included)
    auto range = [&](uint32_t k, int a, int64_t& i0, int64_t& i1) {
        const double c = L[4 * k + a], r = fabs(L[4 * k + 3]);
        const double pad = 1e-3 * g.cell[a] + 4e-6 * (fabs(c) + r);
        i0 = (int64_t)floor((c - r - pad - g.lo[a]) / g.cell[a]);
        i1 = (int64_t)floor((c + r + pad - g.lo[a]) / g.cell[a]);
        i0 = std::max<int64_t>(0, std::min<int64_t>(i0, (int64_t)g.n[a] - 1));
        i1 = std::max<int64_t>(0, std::min<int64_t>(i1, (int64_t)g.n[a] - 1));
    };
    // pass 0 sizes the grid over every finite light and sends the lights that
    // span too many cells to the big list; pass 1 sizes it over the rest
    for (int pass = 0; pass < 2; ++pass) {
        double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
        uint32_t m = 0;
        for (uint32_t k = 0; k < n; ++k) {
            if (big[k]) continue;
            const double r = fabs(L[4 * k + 3]);
            for (int a = 0; a < 3; ++a) {
                lo[a] = std::min(lo[a], L[4 * k + a] - r);
                hi[a] = std::max(hi[a], L[4 * k + a] + r);
            }
            ++m;
        }
        if (m == 0) {
            g = LightGrid{};
            break;
        }
        double scale = 0.0, e[3];
        for (int a = 0; a < 3; ++a) scale = std::max(scale, std::max(fabs(lo[a]), fabs(hi[a])));
        for (int a = 0; a < 3; ++a) {
            const double pb = 1e-4 * (hi[a] - lo[a]) + 1e-5 * scale + 1e-6;
            lo[a] -= pb;
            hi[a] += pb;
            e[a] = hi[a] - lo[a];
        }
        // cubic cells of side h with ~cells_per_light * m cells; an extent
        // thinner than h gets one cell and h is re-solved over the others
        const double target = std::max(1.0, cells_per_light * m);
        bool flat[3] = {false, false, false};
        double h = std::max(e[0], std::max(e[1], e[2]));
        for (int it = 0; it < 3; ++it) {
            double vol = 1.0;
            int dims = 0;
            for (int a = 0; a < 3; ++a)
                if (!flat[a]) {
                    vol *= e[a];
                    ++dims;
                }
            if (dims == 0) break;
            h = pow(vol / target, 1.0 / dims);
            bool changed = false;
            for (int a = 0; a < 3; ++a)
                if (!flat[a] && e[a] < h) flat[a] = changed = true;
            if (!changed) break;
        }
        for (;;) {
            uint64_t cells = 1;
            for (int a = 0; a < 3; ++a) {
                g.n[a] = flat[a] ? 1u : (uint32_t)std::min(4096.0, std::max(1.0, ceil(e[a] / h)));
                cells *= g.n[a];
            }
            if (cells <= (1u << 24)) break;
            h *= 1.25;
        }
        for (int a = 0; a < 3; ++a) {
            g.lo[a] = lo[a];
            g.cell[a] = e[a] / g.n[a];
        }
        if (pass == 0)
            for (uint32_t k = 0; k < n; ++k) {
                if (big[k]) continue;
                uint64_t span = 1;
                for (int a = 0; a < 3; ++a) {
                    int64_t i0, i1;
                    range(k, a, i0, i1);
                    span *= (uint64_t)(i1 - i0 + 1);
                }
                if (span > kGridBigCells) big[k] = 1;
            }
    }
    const uint64_t cells = (uint64_t)g.n[0] * g.n[1] * g.n[2];
    auto each_cell = [&](uint32_t k, auto&& f) {
        int64_t i0[3], i1[3];
        for (int a = 0; a < 3; ++a) range(k, a, i0[a], i1[a]);
        for (int64_t z = i0[2]; z <= i1[2]; ++z)
            for (int64_t y = i0[1]; y <= i1[1]; ++y)
                for (int64_t x = i0[0]; x <= i1[0]; ++x) f((uint64_t)((z * g.n[1] + y) * g.n[0] + x));
    };
    std::vector<uint32_t> cnt(cells, 0);
    for (uint32_t k = 0; k < n; ++k)
        if (big[k]) ++g.n_big;
        else each_cell(k, [&](uint64_t c) { ++cnt[c]; });
    g.start.assign(cells + 1, g.n_big);
    for (uint64_t c = 0; c < cells; ++c) g.start[c + 1] = g.start[c] + cnt[c];
    g.items.assign(g.start[cells], 0);
    std::vector<uint32_t> fill(g.start.begin(), g.start.end() - 1);
    uint32_t q = 0;
    for (uint32_t k = 0; k < n; ++k)
        if (big[k]) g.items[q++] = k;
        else each_cell(k, [&](uint64_t c) { g.items[fill[c]++] = k; });
    return g;
}


std::vector<float> light_grid_records(const LightGrid& g, const double* L, bool abs_radius) {
    const size_t n_cells = g.start.empty() ? 0 : g.start.size() - 1;
    constexpr uint32_t S = kGridRecSlots;
    auto fbits = [](uint32_t u) {
        float f;
        memcpy(&f, &u, 4);
        return f;
    };
    const float qnan = fbits(0x7fc00000u);
    std::vector<float> rec(n_cells * S * 4, qnan);
    for (size_t c = 0; c < n_cells; ++c) {
        const uint32_t lo = g.start[c], n = g.start[c + 1] - lo;
        float* r = rec.data() + c * S * 4;
        const uint32_t inl = n <= S ? n : S - 1;
        for (uint32_t i = 0; i < inl; ++i) {
            const double* l = L + 4 * (size_t)g.items[lo + i];
            r[4 * i + 0] = (float)l[0];
            r[4 * i + 1] = (float)l[1];
            r[4 * i + 2] = (float)l[2];
            r[4 * i + 3] = abs_radius ? fabsf((float)l[3]) : (float)l[3];
        }
        if (n > S) {
            r[4 * (S - 1) + 0] = fbits(lo + inl);
            r[4 * (S - 1) + 1] = fbits(n - inl);
            r[4 * (S - 1) + 2] = fbits(kGridRecLink);
        }
    }
    return rec;
}

}  // namespace rtw
