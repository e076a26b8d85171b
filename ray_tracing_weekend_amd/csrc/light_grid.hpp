// light_grid.hpp -- the light grid's cell walk (the light pdf's all-hits
// query over long light lists, render_kernel.hpp lights_pdf_grid).  Host +
// device: tests/native/grid_walk_check.cpp runs the f64 instance on the CPU
// against a brute-force sweep (every hit light counted exactly once), whole
// and cut into pieces as the wave-cooperative walk cuts it.
#pragma once

#include <math.h>
#include <stdint.h>

#include "host/bvh.hpp"
#include "rtw_device.hpp"
#include "rtw_kernels.h"

namespace rtw {
namespace dev {

// 1 / x as the render kernels compute it (f32: the hardware reciprocal)
__host__ __device__ inline double grid_inv(double x) { return 1.0 / x; }
__device__ inline float grid_inv(float x) { return __builtin_amdgcn_rcpf(x); }

// Light pdf through the light grid (KParams::light_bvh == 2; host/bvh.hpp
// LightGrid): a 3-D DDA walks the cells the ray (o, d), t in [0, inf), crosses
// and calls item(k, te, tx) for every light listed in a cell, with [te, tx)
// the ray-parameter interval the walk assigns to that cell.  The intervals
// partition the real line (the first starts at -inf, the last ends at +inf,
// each ends where the next starts, never decreasing), so a light counted only
// where its closest-approach parameter falls is counted at most once however
// the walk rounds; the host pads every light's cell range by more than that
// rounding, so a hit light is counted exactly once.  (Fetching the next
// cells' ranges ahead of the tests measured slower: C5 +3 % to +15 % time.)
// `ncell` (may be null): += the cells visited (KParams::counters[8]).
template <typename R, typename Item>
__host__ __device__ inline void light_grid_walk(const DevScene<R>& sc, V3<R> o, V3<R> d, Item&& item,
                                                uint32_t* ncell = nullptr) {
    const R kInf = (R)INFINITY;
    const R ix = grid_inv(d.x), iy = grid_inv(d.y), iz = grid_inv(d.z);
    R tn, tf;
    {
        const R x0 = (sc.lg_lo[0] - o.x) * ix, x1 = (sc.lg_hi[0] - o.x) * ix;
        const R y0 = (sc.lg_lo[1] - o.y) * iy, y1 = (sc.lg_hi[1] - o.y) * iy;
        const R z0 = (sc.lg_lo[2] - o.z) * iz, z1 = (sc.lg_hi[2] - o.z) * iz;
        tn = fmax(fmax(fmin(x0, x1), fmin(y0, y1)), fmax(fmin(z0, z1), (R)0));
        tf = fmin(fmax(x0, x1), fmin(fmax(y0, y1), fmax(z0, z1)));
    }
    if (!(tn <= tf)) return;
    const int nx = (int)sc.lg_n[0], ny = (int)sc.lg_n[1], nz = (int)sc.lg_n[2];
    // the entry cell (clamped; NaN -> 0)
    auto cell_of = [&](R oc, R dc, R lo, R inv, int n) {
        return (int)fmin(fmax((oc + tn * dc - lo) * inv, (R)0), (R)(n - 1));
    };
    int cx = cell_of(o.x, d.x, sc.lg_lo[0], sc.lg_inv[0], nx);
    int cy = cell_of(o.y, d.y, sc.lg_lo[1], sc.lg_inv[1], ny);
    int cz = cell_of(o.z, d.z, sc.lg_lo[2], sc.lg_inv[2], nz);
    const int sx = d.x > 0 ? 1 : (d.x < 0 ? -1 : 0);
    const int sy = d.y > 0 ? 1 : (d.y < 0 ? -1 : 0);
    const int sz = d.z > 0 ? 1 : (d.z < 0 ? -1 : 0);
    R te = -kInf;
    // where the ray leaves cell c along one axis (+inf: never), not before te
    auto exit_t = [&](int c, int s, R lo, R cell, R oc, R inv) {
        return s == 0 ? kInf : fmax((lo + (R)(c + (s > 0 ? 1 : 0)) * cell - oc) * inv, te);
    };
    R tmx = exit_t(cx, sx, sc.lg_lo[0], sc.lg_cell[0], o.x, ix);
    R tmy = exit_t(cy, sy, sc.lg_lo[1], sc.lg_cell[1], o.y, iy);
    R tmz = exit_t(cz, sz, sc.lg_lo[2], sc.lg_cell[2], o.z, iz);
    uint32_t c = (uint32_t)((cz * ny + cy) * nx + cx);
    for (;;) {
        int axis, ni, nn;
        R tx;
        if (tmx <= tmy && tmx <= tmz) {
            axis = 0; tx = tmx; ni = cx + sx; nn = nx;
        } else if (tmy <= tmz) {
            axis = 1; tx = tmy; ni = cy + sy; nn = ny;
        } else {
            axis = 2; tx = tmz; ni = cz + sz; nn = nz;
        }
        const bool last = !(tx < kInf) || ni < 0 || ni >= nn;
        if (last) tx = kInf;
        const uint32_t b = sc.lg_start[c], e = sc.lg_start[c + 1];
        if (ncell) ++*ncell;
        for (uint32_t k = b; k < e; ++k) item(k, te, tx);
        if (last) break;
        te = tx;
        if (axis == 0) {
            cx = ni;
            c += sx;
            tmx = exit_t(cx, sx, sc.lg_lo[0], sc.lg_cell[0], o.x, ix);
        } else if (axis == 1) {
            cy = ni;
            c += sy * nx;
            tmy = exit_t(cy, sy, sc.lg_lo[1], sc.lg_cell[1], o.y, iy);
        } else {
            cz = ni;
            c += sz * nx * ny;
            tmz = exit_t(cz, sz, sc.lg_lo[2], sc.lg_cell[2], o.z, iz);
        }
    }
}

// The grid interval [tn, tf] of the ray (the box clip light_grid_walk starts
// from) and the number of cells the walk crosses in it (entry and exit cells
// of the clip, one step per crossed cell boundary); false: the ray misses the
// grid.  Used to cut a walk into pieces (lights_pdf_grid_coop).
template <typename R>
__host__ __device__ inline bool light_grid_span(const DevScene<R>& sc, V3<R> o, V3<R> d, R ix, R iy, R iz, R& tn, R& tf,
                                       uint32_t& cells) {
    const R x0 = (sc.lg_lo[0] - o.x) * ix, x1 = (sc.lg_hi[0] - o.x) * ix;
    const R y0 = (sc.lg_lo[1] - o.y) * iy, y1 = (sc.lg_hi[1] - o.y) * iy;
    const R z0 = (sc.lg_lo[2] - o.z) * iz, z1 = (sc.lg_hi[2] - o.z) * iz;
    tn = fmax(fmax(fmin(x0, x1), fmin(y0, y1)), fmax(fmin(z0, z1), (R)0));
    tf = fmin(fmax(x0, x1), fmin(fmax(y0, y1), fmax(z0, z1)));
    if (!(tn <= tf)) return false;
    auto span = [&](R oc, R dc, R lo, R inv, int n) {
        const int a = (int)fmin(fmax((oc + tn * dc - lo) * inv, (R)0), (R)(n - 1));
        const int b = (int)fmin(fmax((oc + tf * dc - lo) * inv, (R)0), (R)(n - 1));
        return (uint32_t)(a > b ? a - b : b - a);
    };
    cells = 1u + span(o.x, d.x, sc.lg_lo[0], sc.lg_inv[0], (int)sc.lg_n[0]) +
            span(o.y, d.y, sc.lg_lo[1], sc.lg_inv[1], (int)sc.lg_n[1]) +
            span(o.z, d.z, sc.lg_lo[2], sc.lg_inv[2], (int)sc.lg_n[2]);
    return true;
}

// One piece of light_grid_walk: the cells the ray crosses from t0 on, with the
// walk's interval bookkeeping clipped to the piece -- the first interval
// starts at t0 (-inf for the ray's first piece, `head`), and the cell the walk
// is in when it passes t1 ends the piece at t1 (+inf for the ray's last piece,
// `tail`).  The pieces [t_j, t_j+1) of one ray partition the real line as the
// whole walk's intervals do, so a light is counted at most once over them; a
// piece finds its entry cell as the whole walk does (the point at t0, clamped
// into the grid: the same rounding, covered by the host's padding), so a hit
// light is counted exactly once.  head && tail with t0 = tn is light_grid_walk.
// cell(c, te, tx) is called for every cell c of the piece with its interval.
template <typename R, typename Cell>
__host__ __device__ inline void light_grid_walk_cells(const DevScene<R>& sc, V3<R> o, V3<R> d, R ix, R iy, R iz, R t0,
                                                      R t1, bool head, bool tail, Cell&& cell) {
    const R kInf = (R)INFINITY;
    const int nx = (int)sc.lg_n[0], ny = (int)sc.lg_n[1], nz = (int)sc.lg_n[2];
    auto cell_of = [&](R oc, R dc, R lo, R inv, int n) {
        return (int)fmin(fmax((oc + t0 * dc - lo) * inv, (R)0), (R)(n - 1));
    };
    int cx = cell_of(o.x, d.x, sc.lg_lo[0], sc.lg_inv[0], nx);
    int cy = cell_of(o.y, d.y, sc.lg_lo[1], sc.lg_inv[1], ny);
    int cz = cell_of(o.z, d.z, sc.lg_lo[2], sc.lg_inv[2], nz);
    const int sx = d.x > 0 ? 1 : (d.x < 0 ? -1 : 0);
    const int sy = d.y > 0 ? 1 : (d.y < 0 ? -1 : 0);
    const int sz = d.z > 0 ? 1 : (d.z < 0 ? -1 : 0);
    R te = head ? -kInf : t0;
    auto exit_t = [&](int c, int s, R lo, R cell, R oc, R inv) {
        return s == 0 ? kInf : fmax((lo + (R)(c + (s > 0 ? 1 : 0)) * cell - oc) * inv, te);
    };
    R tmx = exit_t(cx, sx, sc.lg_lo[0], sc.lg_cell[0], o.x, ix);
    R tmy = exit_t(cy, sy, sc.lg_lo[1], sc.lg_cell[1], o.y, iy);
    R tmz = exit_t(cz, sz, sc.lg_lo[2], sc.lg_cell[2], o.z, iz);
    uint32_t c = (uint32_t)((cz * ny + cy) * nx + cx);
    for (;;) {
        int axis, ni, nn;
        R tx;
        if (tmx <= tmy && tmx <= tmz) {
            axis = 0; tx = tmx; ni = cx + sx; nn = nx;
        } else if (tmy <= tmz) {
            axis = 1; tx = tmy; ni = cy + sy; nn = ny;
        } else {
            axis = 2; tx = tmz; ni = cz + sz; nn = nz;
        }
        const bool last = !(tx < kInf) || ni < 0 || ni >= nn;
        bool stop = last;
        if (!tail) {
            if (last || !(tx < t1)) {
                tx = t1;
                stop = true;
            }
        } else if (last) {
            tx = kInf;
        }
        cell(c, te, tx);
        if (stop) break;
        te = tx;
        if (axis == 0) {
            cx = ni;
            c += sx;
            tmx = exit_t(cx, sx, sc.lg_lo[0], sc.lg_cell[0], o.x, ix);
        } else if (axis == 1) {
            cy = ni;
            c += sy * nx;
            tmy = exit_t(cy, sy, sc.lg_lo[1], sc.lg_cell[1], o.y, iy);
        } else {
            cz = ni;
            c += sz * nx * ny;
            tmz = exit_t(cz, sz, sc.lg_lo[2], sc.lg_cell[2], o.z, iz);
        }
    }
}

// light_grid_walk_cells with item(k, te, tx) for every light k listed in a
// visited cell (two dependent loads per cell: the cell's range, then its
// lights)
template <typename R, typename Item>
__host__ __device__ inline void light_grid_walk_piece(const DevScene<R>& sc, V3<R> o, V3<R> d, R ix, R iy, R iz, R t0, R t1,
                                             bool head, bool tail, Item&& item, uint32_t* ncell = nullptr) {
    light_grid_walk_cells(sc, o, d, ix, iy, iz, t0, t1, head, tail, [&](uint32_t c, R te, R tx) {
        const uint32_t b = sc.lg_start[c], e = sc.lg_start[c + 1];
        if (ncell) ++*ncell;
        for (uint32_t k = b; k < e; ++k) item(k, te, tx);
    });
}

// Cell records (DevScene::lg_rec, staged by the host with the grid): per cell
// kGridRecSlots f32 lights {c, r} as the f32 walk reads them (the f32
// kernels' lg_sph, the f64 kernels' lg_sph32), so a visited cell costs ONE
// 64-byte load instead of the range load and then one load per light.  A cell
// of n <= 4 lights holds them in slots 0..n-1 and all-NaN slots after them (a
// NaN light fails every test: each is a conjunction of comparisons); a cell of
// n > 4 holds its first 3 and, in slot 3, a link {start bits, count bits, z
// bits kGridRecLink, NaN} to the rest of its list in lg_sph (a link fails
// every test too: its z is NaN).
__host__ __device__ inline uint32_t grid_rec_bits(float x) { return __builtin_bit_cast(uint32_t, x); }

// light_grid_walk_cells over the cell records: item(L, idx, te, tx) for every
// slot of a visited cell (the empty ones included: NaN) and every linked
// light, with L the f32 light and idx() its position in lg_sph / lg_id (for
// an inline slot a load of the cell's range start: call it for candidates
// only).  `items`: the f32 lights of lg_sph's order (the links' targets).
// ncell / ntest (may be null): += the cells visited / the lights listed in
// them.
template <typename R, typename Item>
__host__ __device__ inline void light_grid_walk_piece_rec(const DevScene<R>& sc, const R4<float>* __restrict__ rec,
                                                          const R4<float>* __restrict__ items, V3<R> o, V3<R> d, R ix,
                                                          R iy, R iz, R t0, R t1, bool head, bool tail, Item&& item,
                                                          uint32_t* ncell = nullptr, uint32_t* ntest = nullptr) {
    auto tests = [&](uint32_t c, R te, R tx, const R4<float>& s0, const R4<float>& s1, const R4<float>& s2,
                     const R4<float>& s3) {
        const bool link = grid_rec_bits(s3.z) == kGridRecLink;
        const uint32_t lb = grid_rec_bits(s3.x), ln = link ? grid_rec_bits(s3.y) : 0u;
        if (ncell) ++*ncell;
        if (ntest) *ntest += (s0.w == s0.w) + (s1.w == s1.w) + (s2.w == s2.w) + (s3.w == s3.w) + ln;
        item(s0, [&]() { return sc.lg_start[c]; }, te, tx);
        item(s1, [&]() { return sc.lg_start[c] + 1u; }, te, tx);
        item(s2, [&]() { return sc.lg_start[c] + 2u; }, te, tx);
        item(s3, [&]() { return sc.lg_start[c] + 3u; }, te, tx);
        for (uint32_t q = lb; q < lb + ln; ++q) item(items[q], [q]() { return q; }, te, tx);
    };
#if RTW_GRID_PF
    // one cell ahead: a cell's record is loaded before the previous cell's
    // tests run, so two of a lane's record loads are in flight
    bool have = false;
    uint32_t pc = 0;
    R pte = 0, ptx = 0;
    R4<float> p0{}, p1{}, p2{}, p3{};
    light_grid_walk_cells(sc, o, d, ix, iy, iz, t0, t1, head, tail, [&](uint32_t c, R te, R tx) {
        const R4<float>* r = rec + (size_t)kGridRecSlots * c;
        const R4<float> s0 = r[0], s1 = r[1], s2 = r[2], s3 = r[3];
        if (have) tests(pc, pte, ptx, p0, p1, p2, p3);
        have = true;
        pc = c;
        pte = te;
        ptx = tx;
        p0 = s0;
        p1 = s1;
        p2 = s2;
        p3 = s3;
    });
    if (have) tests(pc, pte, ptx, p0, p1, p2, p3);
#else
    light_grid_walk_cells(sc, o, d, ix, iy, iz, t0, t1, head, tail, [&](uint32_t c, R te, R tx) {
        const R4<float>* r = rec + (size_t)kGridRecSlots * c;
        const R4<float> s0 = r[0], s1 = r[1], s2 = r[2], s3 = r[3];
        tests(c, te, tx, s0, s1, s2, s3);
    });
#endif
}

}  // namespace dev
}  // namespace rtw
