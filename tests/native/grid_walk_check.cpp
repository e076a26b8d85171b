// grid_walk_check.cpp -- CPU check of the light grid (host/bvh.cpp
// build_light_grid + light_grid.hpp light_grid_walk, the f64 instance the
// parity kernels run): for random light sets and random rays, the walk's
// closest-approach rule must count every light the ray hits exactly once and
// no light twice; the cell-record walk (light_grid_walk_piece_rec, the
// kernels' cooperative walks) must visit exactly the range walk's lights and
// intervals.  Built and run by tests/test_light_grid_host.py:
//   hipcc -x hip --cuda-host-only -O2 -std=c++17 -I<csrc> -I<include> \
//       grid_walk_check.cpp <csrc>/host/bvh.cpp -o grid_walk_check
#include <stdio.h>

#include <algorithm>
#include <random>
#include <tuple>
#include <vector>

#include "host/bvh.hpp"
#include "light_grid.hpp"

using rtw::R4;
using V = rtw::dev::V3<double>;

// ray t >= 0 vs sphere: -1 miss, 1 hit, 0 too close to tangent to call
static int hit_class(const double* L, V o, V d) {
    const double fx = o.x - L[0], fy = o.y - L[1], fz = o.z - L[2];
    const double a = d.x * d.x + d.y * d.y + d.z * d.z;
    const double hb = d.x * fx + d.y * fy + d.z * fz;
    const double c = fx * fx + fy * fy + fz * fz - L[3] * L[3];
    const double disc = hb * hb - a * c;
    const double scale = hb * hb + fabs(a * c) + 1e-300;
    if (disc < -1e-9 * scale) return -1;
    if (disc < 1e-9 * scale) return 0;
    const double far = (-hb + sqrt(disc)) / a;
    if (far < -1e-9 * (fabs(hb) / a + 1.0)) return -1;
    if (far < 1e-9 * (fabs(hb) / a + 1.0)) return 0;
    return 1;
}

int main() {
    std::mt19937_64 rng(12345);
    std::uniform_real_distribution<double> U(0.0, 1.0);
    long checked = 0, hits = 0, bad = 0, rec_visits = 0;
    for (int scene = 0; scene < 6; ++scene) {
        // 0: a field of small lights in a thin layer + one large light (the
        // scenes::simple shape); 1: random sizes in a box; 2: coincident
        // centres and zero radii; 3: a few lights; 4: one huge light among
        // small ones; 5: non-finite entries
        const uint32_t n = scene == 3 ? 5 : 2000;
        std::vector<double> L(4 * n);
        for (uint32_t k = 0; k < n; ++k) {
            double* l = &L[4 * k];
            switch (scene) {
            case 0: l[0] = -50 + 100 * U(rng); l[1] = 0.2; l[2] = -50 + 100 * U(rng); l[3] = 0.2; break;
            case 1: for (int a = 0; a < 3; ++a) l[a] = -10 + 20 * U(rng); l[3] = 0.05 + 0.5 * U(rng); break;
            case 2: l[0] = (k % 7) * 0.5; l[1] = 1.0; l[2] = (k % 3) * 0.5; l[3] = (k % 5) ? 0.3 : 0.0; break;
            case 3: for (int a = 0; a < 3; ++a) l[a] = -3 + 6 * U(rng); l[3] = 0.5 + U(rng); break;
            case 4: for (int a = 0; a < 3; ++a) l[a] = -20 + 40 * U(rng); l[3] = 0.1 + 0.2 * U(rng); break;
            default: for (int a = 0; a < 3; ++a) l[a] = -5 + 10 * U(rng); l[3] = 0.2 + 0.3 * U(rng); break;
            }
            if (scene == 1 && k % 9 == 0) l[3] = -l[3];   // negative radius: same ball
        }
        if (scene == 0) { L[0] = 0; L[1] = 1; L[2] = 0; L[3] = 1.0; }
        if (scene == 4) { L[4] = 0; L[5] = 0; L[6] = 0; L[7] = 30.0; }
        if (scene == 5) { L[3] = INFINITY; L[4 * 7 + 1] = NAN; }
        for (double density : {1.0 / 16, 0.25, 2.0, 16.0}) {
            const rtw::LightGrid g = rtw::build_light_grid(L.data(), n, density);
            std::vector<R4<double>> items(g.items.size());
            for (size_t q = 0; q < g.items.size(); ++q) {
                const double* l = &L[4 * g.items[q]];
                items[q] = R4<double>{l[0], l[1], l[2], l[3]};
            }
            // the cell records of the f32 walk (light_grid_walk_piece_rec), radius as given
            const std::vector<float> recf = rtw::light_grid_records(g, L.data(), false);
            std::vector<R4<float>> items32(g.items.size());
            for (size_t q = 0; q < g.items.size(); ++q) {
                const double* l = &L[4 * g.items[q]];
                items32[q] = R4<float>{(float)l[0], (float)l[1], (float)l[2], (float)l[3]};
            }
            const R4<float>* rec = reinterpret_cast<const R4<float>*>(recf.data());
            rtw::DevScene<double> sc{};
            sc.lg_start = g.start.data();
            sc.lg_sph = items.data();
            sc.lg_id = g.items.data();
            for (int a = 0; a < 3; ++a) {
                sc.lg_lo[a] = g.lo[a];
                sc.lg_hi[a] = g.lo[a] + g.n[a] * g.cell[a];
                sc.lg_cell[a] = g.cell[a];
                sc.lg_inv[a] = 1.0 / g.cell[a];
                sc.lg_n[a] = g.n[a];
            }
            sc.lg_big = g.n_big;
            std::vector<int> count(n);
            for (int r = 0; r < 3000; ++r) {
                // origins on or near light surfaces and in the open; grazing
                // and axis-aligned directions included
                V o, d;
                const uint32_t t = (uint32_t)(U(rng) * n);
                const double* lt = &L[4 * t];
                if (r % 3 == 0 && std::isfinite(lt[0] + lt[1] + lt[2] + lt[3])) {
                    o = V{lt[0] + lt[3], lt[1], lt[2]};
                } else {
                    o = V{-60 + 120 * U(rng), -1 + 4 * U(rng), -60 + 120 * U(rng)};
                }
                if (r % 5 == 0) {
                    const double* tg = &L[4 * (uint32_t)(U(rng) * n)];
                    d = V{tg[0] - o.x, tg[1] - o.y, tg[2] - o.z};
                } else {
                    d = V{-1 + 2 * U(rng), (-1 + 2 * U(rng)) * (r % 2 ? 0.01 : 1.0), -1 + 2 * U(rng)};
                }
                if (r % 17 == 0) d = V{1, 0, 0};
                if (r % 19 == 0) d = V{0, 0, -2};
                if (!std::isfinite(d.x + d.y + d.z)) continue;   // aimed at a NaN light
                std::fill(count.begin(), count.end(), 0);
                for (uint32_t q = 0; q < g.n_big; ++q) ++count[g.items[q]];
                const double ia = 1.0 / (d.x * d.x + d.y * d.y + d.z * d.z);
                rtw::dev::light_grid_walk(sc, o, d, [&](uint32_t q, double te, double tx) {
                    const R4<double>& l = items[q];
                    const double tc = -((o.x - l.x) * d.x + (o.y - l.y) * d.y + (o.z - l.z) * d.z) * ia;
                    if (tc >= te && tc < tx && hit_class(&L[4 * g.items[q]], o, d) >= 0) ++count[g.items[q]];
                });
                // the same walk cut into pieces (render_kernel.hpp lights_pdf_grid_coop):
                // k = ceil(cells / P) pieces of equal length in t
                std::vector<int> pc(3 * n, 0);
                {
                    const double ix = rtw::dev::grid_inv(d.x), iy = rtw::dev::grid_inv(d.y), iz = rtw::dev::grid_inv(d.z);
                    double tn, tf;
                    uint32_t cells = 0;
                    const uint32_t Ps[3] = {1, 3, 8};
                    if (rtw::dev::light_grid_span(sc, o, d, ix, iy, iz, tn, tf, cells)) {
                        for (int v = 0; v < 3; ++v) {
                            const uint32_t kp = (cells + Ps[v] - 1) / Ps[v];
                            const double step = (tf - tn) / (double)kp;
                            auto t_at = [&](uint32_t q) { return q == 0 ? tn : fma((double)q, step, tn); };
                            for (uint32_t j = 0; j < kp; ++j) {
                                std::vector<std::tuple<uint32_t, double, double>> seen, seen_rec;
                                uint32_t nc = 0, nc_rec = 0, nt_rec = 0;
                                rtw::dev::light_grid_walk_piece(sc, o, d, ix, iy, iz, t_at(j), t_at(j + 1), j == 0,
                                                                j + 1 == kp, [&](uint32_t q, double te, double tx) {
                                    seen.emplace_back(q, te, tx);
                                    const R4<double>& l = items[q];
                                    const double tc = -((o.x - l.x) * d.x + (o.y - l.y) * d.y + (o.z - l.z) * d.z) * ia;
                                    if (tc >= te && tc < tx && hit_class(&L[4 * g.items[q]], o, d) >= 0)
                                        ++pc[v * n + g.items[q]];
                                }, &nc);
                                // the record walk visits the same (light, interval) pairs, the
                                // empty / link slots as NaN lights, each light as its f32 record
                                rtw::dev::light_grid_walk_piece_rec(sc, rec, items32.data(), o, d, ix, iy, iz, t_at(j),
                                                                    t_at(j + 1), j == 0, j + 1 == kp,
                                                                    [&](const R4<float>& l, auto&& idx, double te, double tx) {
                                    if (!(l.w == l.w)) return;
                                    const uint32_t q = idx();
                                    const R4<float>& w = items32[q];
                                    if (!(l.x == w.x && l.y == w.y && l.z == w.z && l.w == w.w)) ++bad;
                                    seen_rec.emplace_back(q, te, tx);
                                }, &nc_rec, &nt_rec);
                                std::sort(seen.begin(), seen.end());
                                std::sort(seen_rec.begin(), seen_rec.end());
                                if (seen != seen_rec || nc != nc_rec || nt_rec != seen.size()) {
                                    if (bad < 10)
                                        printf("records: scene %d density %g ray %d piece %u: %zu vs %zu visits, %u vs %u cells\n",
                                               scene, density, r, j, seen.size(), seen_rec.size(), nc, nc_rec);
                                    ++bad;
                                }
                                rec_visits += seen.size();
                            }
                        }
                    }
                    for (uint32_t q = 0; q < g.n_big; ++q)
                        for (int v = 0; v < 3; ++v) ++pc[v * n + g.items[q]];
                }
                for (uint32_t k = 0; k < n; ++k) {
                    const int h = hit_class(&L[4 * k], o, d);
                    for (int v = 0; v < 3; ++v) {
                        const bool pok = pc[v * n + k] <= 1 && (h != 1 || pc[v * n + k] == 1);
                        if (!pok && bad < 10)
                            printf("pieces %d: scene %d density %g ray %d light %u: counted %d, hit class %d\n", v,
                                   scene, density, r, k, pc[v * n + k], h);
                        bad += pok ? 0 : 1;
                    }
                    ++checked;
                    if (h == 1) ++hits;
                    const bool ok = count[k] <= 1 && (h != 1 || count[k] == 1);
                    if (!ok && bad < 10)
                        printf("scene %d density %g ray %d light %u: counted %d, hit class %d\n", scene, density, r,
                               k, count[k], h);
                    bad += ok ? 0 : 1;
                }
            }
        }
    }
    printf("checked %ld (ray, light) pairs, %ld hits, %ld wrong; %ld record-walk visits\n", checked, hits, bad,
           rec_visits);
    return bad == 0 && hits > 1000 && rec_visits > 100000 ? 0 : 1;
}
