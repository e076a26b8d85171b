"""BASELINE configs[2] and configs[4] at their configured image size.

C3: the 10k-sphere Lambertian / Metal / Dielectric field (scenes::simple's
generator over a 100 x 100 grid, camera pulled back; 488 light spheres: the
light grid is on), 1920x1080.  C5: the 1M-sphere field (1000 x 1000 grid,
50k light spheres), 1920x1080.  Both render here at their full resolution but
a low spp in the f64 parity mode, and sampled rows are pinned to the oracle
bit for bit (per-pixel MAE < 1e-5, identical NaN masks), as
tests/test_gpu_c4.py does for C4; the f32 speed mode's frame is checked
against the f64 frame statistically.  Generator: scenes/src/lib.rs:155-233,
scaled.
"""
import numpy as np
import pytest

import ray_tracing_weekend_amd as rtw
from oracle import oracle as O

pytestmark = pytest.mark.gpu

SEED_SCENE = 0x5EED0001
W, H, DEPTH = 1920, 1080, 50
F64_MAE_TOL = 1e-5


def _ocam(cam):
    ocam = O.Camera()
    for name, _ in O.Camera._fields_:
        setattr(ocam, name, getattr(cam.raw, name))
    return ocam


def _frame(n, spp, seed, prec):
    soa, b = rtw.scenes.simple_soa(SEED_SCENE, n)
    cam = b.with_image_width(W).with_image_height(H).with_samples_per_pixel(spp).with_max_depth(DEPTH).build()
    with rtw.Renderer(precision=prec) as r:
        r.set_scene(soa)
        img = r.render(cam, seed)
        chunk = int(r.stats.chunk)
        st = r.get_stats()
    return soa, cam, img, chunk, st


@pytest.mark.parametrize("config,n,spp,rows", [
    ("C3", 50, 2, (140, 1080, 310)),
    ("C5", 500, 1, (260, 1080, 400)),
])
def test_full_frame_f64_rows_match_oracle(config, n, spp, rows):
    soa, cam, img, chunk, st = _frame(n, spp, 61, rtw.RTW_F64)
    assert img.shape == (H, W, 3) and st.samples == W * H * spp
    ref, _ = O.render(_ocam(cam), O.Scene(**soa.__dict__), 61, chunk=chunk, accel=O.ACCEL_BVH_CACHED, rows=rows)
    sel = list(range(*rows))
    g, o = img[sel], ref[sel]
    assert np.array_equal(np.isnan(g).any(-1), np.isnan(o).any(-1)), config
    ok = ~np.isnan(o).any(-1)
    assert ok.mean() > 0.5
    assert np.abs(g[ok] - o[ok]).mean() / spp < F64_MAE_TOL and (g[ok] == o[ok]).all(), config


@pytest.mark.parametrize("config,n,spp", [("C3", 50, 8), ("C5", 500, 4)])
def test_full_frame_f32_tracks_f64(config, n, spp):
    """The speed mode's full frame against the parity mode's (other seeds):
    image means within 1 % and the per-row means correlated -- the f32 mode's
    stated tolerance is statistical."""
    _, _, a, _, _ = _frame(n, spp, 71, rtw.RTW_F32)
    _, _, b, _, _ = _frame(n, spp, 73, rtw.RTW_F64)
    ok = ~(np.isnan(a).any(-1) | np.isnan(b).any(-1))
    ma, mb = a[ok].mean(), b[ok].mean()
    assert abs(ma / mb - 1) < 0.01, (config, ma, mb)
    ra = np.nanmean(np.where(ok[..., None], a, np.nan), axis=(1, 2))
    rb = np.nanmean(np.where(ok[..., None], b, np.nan), axis=(1, 2))
    assert np.corrcoef(ra, rb)[0, 1] > 0.99, config


@pytest.mark.parametrize("config,n,spp", [("C3", 50, 4), ("C5", 500, 2)])
def test_cooperative_grid_walk_matches_lane_walk(config, n, spp):
    """The wave-cooperative light-grid walk (grid_piece = P > 0, the default:
    every lane of the wave walks pieces of the pending rays' walks,
    render_kernel.hpp lights_pdf_grid_coop) against one lane per ray
    (grid_piece = 0).  Both count the same lights (the pieces partition the
    walk: tests/native/grid_walk_check.cpp); only the f32 sum of a multi-piece
    ray's pdfs is associated by piece, so the frames agree to f32 rounding,
    NaN masks equal -- and the cut depends on the ray alone, so a render is
    reproduced bit for bit under another scheduling knob."""
    soa, b = rtw.scenes.simple_soa(SEED_SCENE, n)
    cam = b.with_image_width(W).with_image_height(H).with_samples_per_pixel(spp).with_max_depth(DEPTH).build()
    imgs = {}
    for key, tuning in (("coop", {}), ("lane", {"grid_piece": 0}), ("coop_p3", {"grid_piece": 3}),
                        ("coop_pixel_major", {"item_order": 0})):
        with rtw.Renderer(precision=rtw.RTW_F32) as r:
            for k, v in tuning.items():
                r.set_tuning(k, v)
            r.set_scene(soa)
            imgs[key] = r.render(cam, 17)
    c, ln = imgs["coop"], imgs["lane"]
    assert np.array_equal(np.isnan(c).any(-1), np.isnan(ln).any(-1)), config
    ok = ~np.isnan(ln).any(-1)
    assert ok.mean() > 0.5
    rel = np.abs(c[ok] - ln[ok]) / np.maximum(np.abs(ln[ok]), 1e-3)
    assert rel.max() < 1e-3 and rel.mean() < 1e-6, (config, float(rel.max()), float(rel.mean()))
    assert (c[ok] == ln[ok]).mean() > 0.9, config
    same = np.isnan(imgs["coop_pixel_major"]) == np.isnan(c)
    assert same.all() and np.array_equal(np.nan_to_num(imgs["coop_pixel_major"], nan=-7.0), np.nan_to_num(c, nan=-7.0))
    p3 = imgs["coop_p3"]
    assert np.array_equal(np.isnan(p3).any(-1), np.isnan(ln).any(-1))


@pytest.mark.parametrize("config,n,spp", [("C3", 50, 4), ("C5", 500, 2)])
def test_f64_cooperative_grid_walk_is_bit_identical(config, n, spp):
    """f64 (parity mode): the wave-cooperative walk (lights_pdf_grid_coop64:
    the pieces find the hit lights' list indices, each owner sums their pdfs in
    list order) against one lane per ray (grid_piece = 0, lights_pdf_grid) and
    another piece size: the same hit lights, summed in the same order, so the
    frames are equal bit for bit (NaN masks included)."""
    soa, b = rtw.scenes.simple_soa(SEED_SCENE, n)
    cam = b.with_image_width(W).with_image_height(H).with_samples_per_pixel(spp).with_max_depth(DEPTH).build()
    imgs = {}
    for key, tuning in (("coop", {}), ("lane", {"grid_piece": 0}), ("coop_p3", {"grid_piece": 3})):
        with rtw.Renderer(precision=rtw.RTW_F64) as r:
            for k, v in tuning.items():
                r.set_tuning(k, v)
            r.set_scene(soa)
            imgs[key] = r.render(cam, 19)
    ref = np.nan_to_num(imgs["lane"], nan=-7.0)
    for key in ("coop", "coop_p3"):
        assert np.array_equal(np.nan_to_num(imgs[key], nan=-7.0), ref), (config, key)
