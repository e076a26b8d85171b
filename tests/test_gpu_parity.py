"""GPU parity: the HIP render path (through the C-ABI) against the CPU oracle.

f64 (parity mode) must match the oracle to the stated tolerance -- per-pixel
RGB MAE of sum/spp < 1e-5 (BASELINE.json north_star) with identical NaN masks;
the kernel keeps the oracle's operation order, so in practice the pixels are
bit-identical and the test also asserts that.  f32 (speed mode) follows the
same sample paths only until rounding separates them (the reference's
t_min = f64::EPSILON makes self-intersection chaotic), so it is checked
statistically against the f64 oracle.
"""
import numpy as np
import pytest

import ray_tracing_weekend_amd as rtw
from oracle import oracle as O

pytestmark = pytest.mark.gpu

SEED_SCENE = 0x5EED0001
F64_MAE_TOL = 1e-5          # north_star: per-pixel RGB MAE < 1e-5


def _scene(n=11):
    soa, builder = rtw.scenes.simple_soa(SEED_SCENE, n)
    return soa, builder


# render-kernel variants (rtw_stats.kernel)
K_BVH_LOOP, K_BVH_WW, K_BVH4, K_BVH_LDS = 2, 3, 4, 5
BVH_KIND_KERNEL = {0: K_BVH_LOOP, 1: K_BVH_WW, 2: K_BVH4, 3: K_BVH_LDS}
LAST = {}


def _render_gpu(soa, cam, seed, precision, chunk=0, accel=rtw.RTW_ACCEL_AUTO, bvh_kind=None, tuning=None,
                renders=1):
    """renders > 1: the same render repeated by one context (with tuning "lpt"
    the first counts the tile costs, the later ones take the ordered task
    list); every repeat must give the first's image bit for bit."""
    with rtw.Renderer(device=0, precision=precision) as r:
        if chunk:
            r.set_chunk(chunk)
        for k, v in (tuning or {}).items():
            r.set_tuning(k, v)
        if bvh_kind is not None:
            r.set_tuning("bvh_kind", bvh_kind)
        r.set_accel(accel)
        r.set_scene(soa)
        img = r.render(cam, seed)
        for _ in range(renders - 1):
            again = r.render(cam, seed)
            assert _same(img, again)
        LAST["kernel"] = r.stats.kernel
        if bvh_kind is not None:
            # bvh_kind 3 falls back to 1 when the tree does not fit in LDS
            assert r.stats.kernel == BVH_KIND_KERNEL[bvh_kind] or (bvh_kind == 3 and r.stats.kernel == K_BVH_WW)
        return img, r.stats.chunk, (r.stats.segments, r.stats.lambertian)


def _render_oracle(soa, cam, seed, chunk, accel=None):
    ocam = O.Camera()
    for name, _ in O.Camera._fields_:
        setattr(ocam, name, getattr(cam.raw, name))
    img, st = O.render(ocam, O.Scene(**soa.__dict__), seed, chunk=chunk,
                       accel=O.ACCEL_BVH_CACHED if accel is None else accel)
    return img, st


def _compare_f64(gpu, ref, spp):
    nan_g, nan_r = np.isnan(gpu).any(-1), np.isnan(ref).any(-1)
    assert np.array_equal(nan_g, nan_r), f"NaN masks differ: {nan_g.sum()} vs {nan_r.sum()}"
    ok = ~nan_r
    mae = float(np.abs(gpu[ok] - ref[ok]).mean() / spp) if ok.any() else 0.0
    exact = float((gpu == ref).all(-1)[ok].mean()) if ok.any() else 1.0
    return mae, exact


@pytest.mark.parametrize("w,h,spp,depth,chunk", [
    (48, 32, 8, 50, 0),       # auto chunk
    (37, 21, 5, 50, 2),       # ragged tiles, several chunks, last chunk partial
    (3, 2, 10, 3, 0),         # integration-tests small_test geometry (lib.rs:28-49)
    (16, 16, 4, 1, 0),        # depth 1: primary rays only
])
def test_f64_matches_oracle(w, h, spp, depth, chunk):
    soa, b = _scene()
    cam = b.with_image_width(w).with_image_height(h).with_samples_per_pixel(spp) \
           .with_max_depth(depth).build()
    gpu, used_chunk, (segs, lambs) = _render_gpu(soa, cam, 11, rtw.RTW_F64, chunk)
    ref, st = _render_oracle(soa, cam, 11, used_chunk)
    mae, exact = _compare_f64(gpu, ref, spp)
    assert mae < F64_MAE_TOL
    assert exact > 0.999, f"only {exact:.4f} of the pixels are bit-identical"
    assert segs == st.segments and lambs == st.lambertian


def test_f64_small_test_camera():
    """integration-tests small_test (lib.rs:28-49): 3x2, 10 spp, depth 3, its own camera."""
    soa, _ = _scene()
    cam = rtw.CameraBuilder().with_image_width(3).with_image_height(2).with_samples_per_pixel(10) \
        .with_max_depth(3).with_lookfrom((-13, 2, 3)).with_lookat((0, 0, 0)) \
        .with_vup((0, 1, 0)).with_focus_dist(10.0).build()
    gpu, chunk, _ = _render_gpu(soa, cam, 3, rtw.RTW_F64)
    ref, _ = _render_oracle(soa, cam, 3, chunk)
    mae, exact = _compare_f64(gpu, ref, 10)
    assert mae < F64_MAE_TOL and exact == 1.0


def test_max_depth_zero_is_black():
    soa, b = _scene()
    cam = b.with_image_width(9).with_image_height(9).with_samples_per_pixel(3).with_max_depth(0).build()
    for prec in (rtw.RTW_F32, rtw.RTW_F64):
        gpu, _, (segs, _) = _render_gpu(soa, cam, 1, prec)
        assert np.all(gpu == 0.0) and segs == 0


def test_empty_world_is_background():
    soa = rtw.SceneSoA()
    cam = rtw.CameraBuilder().with_image_width(10).with_image_height(7).with_samples_per_pixel(5) \
        .with_background((0.25, 0.5, 1.0)).build()
    for prec in (rtw.RTW_F32, rtw.RTW_F64):
        gpu, _, _ = _render_gpu(soa, cam, 1, prec)
        np.testing.assert_array_equal(gpu, np.broadcast_to([1.25, 2.5, 5.0], gpu.shape))


def test_lambertian_without_lights_is_an_error():
    """hittable_list.rs:417 panics ('HittableList shouldn't be empty') when a
    Lambertian bounce draws from the empty light list; the render returns
    RTW_E_NO_LIGHTS with the same panic count as the oracle.  A scene whose
    Lambertian surfaces are never hit renders normally."""
    soa = rtw.flatten(rtw.HittableList([rtw.Sphere((0, 0, -1), 0.5, rtw.Lambertian((0.5, 0.5, 0.5)))]),
                      rtw.HittableList())
    cam = rtw.CameraBuilder().with_image_width(8).with_image_height(8).with_samples_per_pixel(4).build()
    ref, st = _render_oracle_allow_panic(soa, cam, 5, 1)
    assert st.panic_no_lights > 0
    for prec in (rtw.RTW_F64, rtw.RTW_F32):
        with rtw.Renderer(precision=prec) as r:
            r.set_scene(soa)
            with pytest.raises(rtw.RenderError) as e:
                r.render(cam, 5)
            assert e.value.code == -3
            if prec == rtw.RTW_F64:
                assert r.stats.panic_no_lights == st.panic_no_lights and r.stats.panic_plane_uv == 0
    away = rtw.CameraBuilder().with_image_width(8).with_image_height(8).with_samples_per_pixel(4) \
        .with_lookat((0, 0, 1)).with_background((0.5, 0.5, 0.5)).build()
    with rtw.Renderer(precision=rtw.RTW_F64) as r:
        r.set_scene(soa)
        np.testing.assert_array_equal(r.render(away, 5), np.full((8, 8, 3), 2.0))


def _render_oracle_allow_panic(soa, cam, seed, chunk, accel=None):
    ocam = O.Camera()
    for name, _ in O.Camera._fields_:
        setattr(ocam, name, getattr(cam.raw, name))
    return O.render(ocam, O.Scene(**soa.__dict__), seed, chunk=chunk,
                    accel=O.ACCEL_BRUTE if accel is None else accel, allow_panic=True)


def test_mixed_materials_custom_scene():
    """A hand-built scene with every in-scope material, a light that a
    Lambertian sphere sits inside (NaN path, sphere.rs:105,121), a tilted
    one-sided plane, and defocus blur on."""
    world = rtw.HittableList()
    # a tilted plane facing down, hit by rays moving down (plane.rs:61-76); its
    # UV takes the rotation branch of get_plane_uv (plane.rs:47-53)
    world.add(rtw.Plane((0, -0.5, 0), (0.1, -1, 0.05), rtw.Lambertian((0.8, 0.8, 0.0))))
    world.add(rtw.Sphere((0, 0, -1.2), 0.5, rtw.Lambertian((0.1, 0.2, 0.5))))
    world.add(rtw.Sphere((-1, 0, -1), 0.5, rtw.Dialectric(1.5)))
    world.add(rtw.Sphere((-1, 0, -1), 0.4, rtw.Dialectric(1 / 1.5)))
    world.add(rtw.Sphere((1, 0, -1), 0.5, rtw.Metal((0.8, 0.6, 0.2), 0.3)))
    world.add(rtw.Sphere((0.3, 0.2, -0.8), 0.1, rtw.INVISIBLE))
    lights = rtw.HittableList([rtw.Sphere((0, 0, -1.2), 0.6), rtw.Sphere((1, 1, 0), 0.2)])
    soa = rtw.flatten(world, lights)
    cam = rtw.CameraBuilder().with_image_width(40).with_image_height(30).with_samples_per_pixel(6) \
        .with_max_depth(20).with_lookfrom((0, 0.3, 1)).with_lookat((0, 0, -1)) \
        .with_defocus_angle(0.05).with_focus_dist(2.0).with_background((0.7, 0.8, 1.0)).build()
    gpu, chunk, _ = _render_gpu(soa, cam, 5, rtw.RTW_F64)
    ref, st = _render_oracle(soa, cam, 5, chunk)
    assert st.nan_samples > 0          # the inside-a-light path is exercised
    mae, exact = _compare_f64(gpu, ref, 6)
    assert mae < F64_MAE_TOL and exact > 0.999


def test_rank_sharding_reassembles_the_image():
    """rtw_render_device over 3 ranks (8x8 tiles, T -> rank T % 3), gathered
    into one buffer and un-interleaved by rtw_assemble_tiles == one full render
    (f64, ragged edge tiles: 50x45); the torch restatement
    (sharding.assemble) gives the same image."""
    import torch
    from ray_tracing_weekend_amd import sharding
    soa, b = _scene()
    cam = b.with_image_width(50).with_image_height(45).with_samples_per_pixel(3).with_max_depth(20).build()
    H, W, N = 45, 50, 3
    full, _, _ = _render_gpu(soa, cam, 9, rtw.RTW_F64)
    with rtw.Renderer(precision=rtw.RTW_F64) as r:
        r.set_scene(soa)
        per = rtw.tiles_for_rank(W, H, 0, N) * 64 * 3
        ranks = torch.full((N, per), -5.0, dtype=torch.float64, device="cuda:0")
        for rank in range(N):
            n = rtw.tiles_for_rank(W, H, rank, N) * 64 * 3
            r.render_device(cam, 9, ranks[rank].data_ptr(), n * 8, rank=rank, nranks=N)
        img = torch.full((H, W, 3), -9.0, dtype=torch.float64, device="cuda:0")
        r.assemble_tiles(ranks.data_ptr(), per * 8, N, W, H, img.data_ptr())
        ref = torch.full_like(img, -9.0)
        sharding.assemble(ref, list(ranks.unbind(0)))
        torch.cuda.synchronize()
    assert np.array_equal(np.nan_to_num(img.cpu().numpy(), nan=-7), np.nan_to_num(full, nan=-7))
    assert torch.equal(torch.nan_to_num(img, nan=-7.0), torch.nan_to_num(ref, nan=-7.0))
    # the packed buffers are what sharding.pack cuts out of the image (padding 0)
    for rank in range(N):
        p = sharding.pack(torch.from_numpy(full), rank, N).reshape(-1)
        got = ranks[rank, : p.numel()].cpu()
        assert torch.equal(torch.nan_to_num(got, nan=-7.0), torch.nan_to_num(p, nan=-7.0))


def test_rank_without_tiles_renders_nothing():
    """More ranks than tiles: a rank with no tiles accepts a NULL d_out and
    renders nothing (a 0-element torch buffer has data_ptr 0)."""
    soa, b = _scene()
    cam = b.with_image_width(8).with_image_height(8).with_samples_per_pixel(2).with_max_depth(5).build()
    assert rtw.tiles_for_rank(8, 8, 1, 2) == 0
    with rtw.Renderer(precision=rtw.RTW_F32) as r:
        r.set_scene(soa)
        r.render_device(cam, 3, 0, 0, rank=1, nranks=2)
        assert r.get_stats().samples == 0



def test_f32_statistically_matches_f64_oracle():
    soa, b = _scene()
    spp = 64
    cam = b.with_image_width(64).with_image_height(36).with_samples_per_pixel(spp).with_max_depth(50).build()
    g32, chunk, _ = _render_gpu(soa, cam, 21, rtw.RTW_F32)
    ref, st = _render_oracle(soa, cam, 21, 0)
    # NaN-free pixels of both: per-image mean radiance within 1% and per-pixel
    # means close to the oracle's in distribution
    ok = ~(np.isnan(g32).any(-1) | np.isnan(ref).any(-1))
    m32, m64 = g32[ok].mean() / spp, ref[ok].mean() / spp
    assert abs(m32 - m64) < 0.01 * m64, (m32, m64)
    d = np.abs(g32[ok] - ref[ok]) / spp
    assert np.median(d) < 0.05
    # NaN pixel fraction within a few points (NaN paths are random events)
    f32n, f64n = np.isnan(g32).any(-1).mean(), np.isnan(ref).any(-1).mean()
    assert abs(f32n - f64n) < 0.05 + 0.5 * f64n


def test_public_render_api_roundtrip(tmp_path):
    world, lights, builder = rtw.scenes.simple(SEED_SCENE)
    cam = builder.with_image_width(20).with_image_height(12).with_samples_per_pixel(2).build()
    sums = cam.render(world, lights, seed=4, precision=rtw.RTW_F64)
    assert sums.shape == (12, 20, 3)
    n = rtw.write_ppm(str(tmp_path / "image.ppm"), sums, 2)
    text = (tmp_path / "image.ppm").read_text().splitlines()
    assert text[:3] == ["P3", "20 12", "255"] and len(text) == 3 + 240 and n > 0


def _same(a, b):
    return np.array_equal(np.nan_to_num(a, nan=-7.0), np.nan_to_num(b, nan=-7.0))


@pytest.mark.parametrize("prec", [rtw.RTW_F32, rtw.RTW_F64])
@pytest.mark.parametrize("n", [11, 14, 30])
@pytest.mark.parametrize("kind", [3, 2, 1, 0])
def test_bvh_equals_brute_force(prec, n, kind):
    """RTW_ACCEL_BVH only culls: the closest hit, hence every pixel, must be
    bit-identical to the brute-force sweep (same per-sphere arithmetic), for
    every traversal (3: binary while-while on the tree staged in LDS, 2: 4-wide
    octant tree, 1: binary while-while, 0: binary single loop)."""
    soa, b = _scene(n)
    cam = b.with_image_width(64).with_image_height(40).with_samples_per_pixel(6).with_max_depth(50).build()
    # the brute-force kernels sum the light pdf linearly; in f32 the light
    # BVH's walk-order sum rounds differently, so it is off here (it has its
    # own test below)
    brute, _, cb = _render_gpu(soa, cam, 13, prec, accel=rtw.RTW_ACCEL_BRUTE)
    bvh, _, cv = _render_gpu(soa, cam, 13, prec, accel=rtw.RTW_ACCEL_BVH, bvh_kind=kind,
                             tuning={"light_bvh_min": 1 << 30})
    if kind == 3 and n == 11:
        assert LAST["kernel"] == K_BVH_LDS          # the C1/C2 scene's tree fits in LDS
    if kind == 3 and n == 14 and prec == rtw.RTW_F64:
        assert LAST["kernel"] == K_BVH_LDS          # 784 spheres: the wide f64 workgroup's LDS (142 KiB)
    assert _same(brute, bvh)
    assert cb == cv


def test_bvh4_stats_and_width():
    soa, b = _scene(11)
    cam = b.with_image_width(48).with_image_height(32).with_samples_per_pixel(4).with_max_depth(50).build()
    with rtw.Renderer(device=0, precision=rtw.RTW_F32) as r:
        r.set_scene(soa)
        r.set_tuning("bvh_kind", 2)
        r.render(cam, 5)
        st = r.stats
        assert st.accel == rtw.RTW_ACCEL_BVH and st.bvh_width == 4
        assert 0 < st.node_visits and 0 < st.sphere_tests
        r.set_tuning("bvh_kind", 1)
        r.render(cam, 5)
        assert r.stats.bvh_width == 2 and r.stats.segments == st.segments


def test_bvh_large_random_scene_equals_brute_force():
    """20k small spheres: deep trees (4-wide stack bound > 13), many leaves
    per ray; f32 BVH must still be bit-identical to brute force."""
    world = rtw.HittableList()
    rng = np.random.default_rng(11)
    mats = [rtw.Lambertian((0.5, 0.5, 0.5)), rtw.Metal((0.8, 0.8, 0.8), 0.1), rtw.Dialectric(1.5)]
    for k in range(20000):
        c = (rng.uniform(-20, 20), rng.uniform(0, 3), rng.uniform(-20, 20))
        world.add(rtw.Sphere(c, float(rng.uniform(0.02, 0.15)), mats[k % 3]))
    world.add(rtw.Plane((0, 0, 0), (0, 1, 0), mats[0]))
    lights = rtw.HittableList([rtw.Sphere((0, 8, 0), 2.0)])
    soa = rtw.flatten(world, lights)
    cam = rtw.CameraBuilder().with_image_width(40).with_image_height(24).with_samples_per_pixel(3) \
        .with_max_depth(20).with_lookfrom((15, 6, 15)).with_lookat((0, 0, 0)).with_vfov(40) \
        .with_background((0.7, 0.8, 1.0)).build()
    brute, _, cb = _render_gpu(soa, cam, 23, rtw.RTW_F32, accel=rtw.RTW_ACCEL_BRUTE)
    bvh, _, cv = _render_gpu(soa, cam, 23, rtw.RTW_F32, accel=rtw.RTW_ACCEL_BVH,
                             tuning={"light_bvh_min": 1 << 30})
    assert _same(brute, bvh) and cb == cv


def test_bvh_f64_matches_oracle_custom_scene():
    world = rtw.HittableList()
    rng = np.random.default_rng(3)
    for k in range(200):
        c = rng.uniform(-3, 3, 3)
        kind = k % 3
        mat = [rtw.Lambertian(rng.uniform(0, 1, 3)), rtw.Metal(rng.uniform(0.5, 1, 3), rng.uniform(0, 0.5)),
               rtw.Dialectric(1.5)][kind]
        world.add(rtw.Sphere(tuple(c), float(rng.uniform(0.05, 0.6)), mat))
    lights = rtw.HittableList([rtw.Sphere((0, 4, 0), 1.0), rtw.Sphere((2, 2, 2), 0.3)])
    soa = rtw.flatten(world, lights)
    cam = rtw.CameraBuilder().with_image_width(32).with_image_height(24).with_samples_per_pixel(4) \
        .with_max_depth(30).with_lookfrom((0, 1, 9)).with_lookat((0, 0, 0)).with_vfov(50) \
        .with_background((0.6, 0.7, 1.0)).build()
    gpu, chunk, _ = _render_gpu(soa, cam, 17, rtw.RTW_F64, accel=rtw.RTW_ACCEL_BVH)
    ref, _ = _render_oracle(soa, cam, 17, chunk)
    mae, exact = _compare_f64(gpu, ref, 4)
    assert mae < F64_MAE_TOL and exact > 0.999


def test_f64_matches_golden_fixtures():
    """The committed golden renders (tests/golden/make_golden.py, oracle at
    fixed seeds): the f64 kernel must reproduce them bit for bit -- the C1
    window (BASELINE configs[0] geometry, 100 spp) and a full 48x27 frame."""
    import json
    import os
    here = os.path.join(os.path.dirname(__file__), "golden")
    with open(os.path.join(here, "simple_scene_5EED0001.json")) as f:
        js = json.load(f)
    soa = rtw.SceneSoA(**{k: np.asarray(js[k], dtype=np.uint32 if k.endswith("mat") or k == "mat_type"
                                        else np.float64) for k in
                          ("spheres", "sphere_mat", "planes", "plane_mat", "mat_type", "mat_params", "lights")})
    gen, builder = rtw.scenes.simple_soa(js["seed"])
    assert np.array_equal(np.asarray(gen.spheres).reshape(-1), np.asarray(soa.spheres).reshape(-1))
    gold = np.load(os.path.join(here, "golden_renders.npz"))
    cases = {"c1_window": (400, 225, 100, (104, 112), (184, 216)),
             "simple_48x27": (48, 27, 16, None, None)}
    for name, (w, h, spp, rows, cols) in cases.items():
        chunk = int(gold[name + "_meta"][0])
        cam = builder.copy().with_image_width(w).with_image_height(h).with_samples_per_pixel(spp) \
            .with_max_depth(50).build()
        img, used, _ = _render_gpu(soa, cam, 0xC0FFEE, rtw.RTW_F64, chunk=chunk)
        assert used == chunk
        if rows is not None:
            img = img[rows[0]:rows[1], cols[0]:cols[1]]
        ref = gold[name]
        mae, exact = _compare_f64(img, ref, spp)
        assert mae < F64_MAE_TOL and exact == 1.0, (name, mae, exact)


def test_partial_buffer_cap_grows_the_chunk():
    """With the chunk-sum buffer capped (tuning "partial_max"), the auto chunk
    grows to fit and the render still matches the oracle at that chunk."""
    soa, b = _scene()
    cam = b.with_image_width(64).with_image_height(64).with_samples_per_pixel(100).with_max_depth(8).build()
    with rtw.Renderer(device=0, precision=rtw.RTW_F64) as r:
        r.set_tuning("partial_max", 1 << 20)     # 64 tiles x 64 px x 3 x 8 B = 96 KiB per chunk
        r.set_scene(soa)
        gpu = r.render(cam, 29)
        chunk = r.stats.chunk
    assert chunk == 10
    ref, _ = _render_oracle(soa, cam, 29, chunk)
    mae, exact = _compare_f64(gpu, ref, 100)
    assert mae < F64_MAE_TOL and exact > 0.999


@pytest.mark.parametrize("prec", [rtw.RTW_F64, rtw.RTW_F32])
def test_light_bvh_equals_linear_light_sum(prec):
    """The light pdf through the light BVH and the light grid at several
    resolutions (tunings light_bvh_min, light_grid) against the linear loop
    over the light list (hittable_list.rs:408-412): f64 sums the hit lights in
    list order, so the images are bit-identical (a light counted twice or
    missed by the grid walk would show); f32 sums in walk order, so only the
    path statistics are compared."""
    world = rtw.HittableList()
    rng = np.random.default_rng(5)
    lights = rtw.HittableList()
    for k in range(300):
        c = (float(rng.uniform(-6, 6)), float(rng.uniform(0.1, 0.4)), float(rng.uniform(-6, 6)))
        r = float(rng.uniform(0.1, 0.3))
        if k % 3 == 0:
            world.add(rtw.Sphere(c, r, rtw.Dialectric(1.5)))
            lights.add(rtw.Sphere(c, r))
        else:
            world.add(rtw.Sphere(c, r, rtw.Lambertian(tuple(rng.uniform(0.2, 0.9, 3)))))
    world.add(rtw.Plane((0, 0, 0), (0, 1, 0), rtw.Lambertian((0.5, 0.5, 0.5))))
    lights.add(rtw.Sphere((1.0, 7.0, -2.0), 3.0))     # spans many grid cells: the grid's big list
    soa = rtw.flatten(world, lights)
    cam = rtw.CameraBuilder().with_image_width(40).with_image_height(24).with_samples_per_pixel(4) \
        .with_max_depth(12).with_lookfrom((8, 3, 8)).with_lookat((0, 0, 0)).with_vfov(45) \
        .with_background((0.7, 0.8, 1.0)).build()
    out = {}
    # light BVH (light_grid 0), light grid at 1/16, 1/4, 1/2 (default) and 16 cells per light, linear loop
    modes = (("bvh", 1, 0), ("grid1", 1, 1), ("grid4", 1, 4), ("grid", 1, 8), ("grid256", 1, 256),
             ("linear", 1 << 30, 8))
    for mode, m, g in modes:
        with rtw.Renderer(device=0, precision=prec) as r:
            r.set_tuning("light_bvh_min", m)
            r.set_tuning("light_grid", g)
            r.set_scene(soa)
            out[mode] = (r.render(cam, 31), r.stats.segments, r.stats.lambertian)
    if prec == rtw.RTW_F64:
        for mode, _, _ in modes[:-1]:
            assert _same(out[mode][0], out["linear"][0]) and out[mode][1:] == out["linear"][1:], mode
        ref, st = _render_oracle(soa, cam, 31, 1)
        mae, exact = _compare_f64(out["grid"][0], ref, 4)
        assert mae < F64_MAE_TOL and exact > 0.999
    else:
        b = out["linear"][0]
        for mode, _, _ in modes[:-1]:
            a = out[mode][0]
            ok = ~(np.isnan(a).any(-1) | np.isnan(b).any(-1))
            assert abs(a[ok].mean() - b[ok].mean()) < 0.02 * b[ok].mean(), mode


# ---- the large-scene configurations of SURVEY.md §8 (C3: 10k spheres, C5: 1M)
# at small image sizes: same scene generator and camera, fewer pixels.

def test_c3_scene_f64_matches_oracle():
    soa, b = rtw.scenes.simple_soa(SEED_SCENE, 50)
    assert len(soa.sphere_mat) > 9000 and len(soa.lights) >= 64     # light BVH on
    cam = b.with_image_width(96).with_image_height(54).with_samples_per_pixel(4).with_max_depth(50).build()
    gpu, chunk, (segs, lambs) = _render_gpu(soa, cam, 41, rtw.RTW_F64)
    ref, st = _render_oracle(soa, cam, 41, chunk)
    mae, exact = _compare_f64(gpu, ref, 4)
    assert mae < F64_MAE_TOL and exact > 0.999
    assert segs == st.segments and lambs == st.lambertian


def test_c5_scene_bvh_equals_brute_force_f32():
    soa, b = rtw.scenes.simple_soa(SEED_SCENE, 500)
    assert len(soa.sphere_mat) > 900_000
    cam = b.with_image_width(24).with_image_height(16).with_samples_per_pixel(2).with_max_depth(20).build()
    off = {"light_bvh_min": 1 << 30}
    brute, _, cb = _render_gpu(soa, cam, 43, rtw.RTW_F32, accel=rtw.RTW_ACCEL_BRUTE, tuning=off)
    bvh, _, cv = _render_gpu(soa, cam, 43, rtw.RTW_F32, accel=rtw.RTW_ACCEL_BVH, tuning=off)
    assert _same(brute, bvh) and cb == cv


def test_c5_scene_f64_matches_oracle():
    soa, b = rtw.scenes.simple_soa(SEED_SCENE, 500)
    cam = b.with_image_width(32).with_image_height(18).with_samples_per_pixel(2).with_max_depth(50).build()
    gpu, chunk, (segs, lambs) = _render_gpu(soa, cam, 47, rtw.RTW_F64)
    ref, st = _render_oracle(soa, cam, 47, chunk)
    mae, exact = _compare_f64(gpu, ref, 2)
    assert mae < F64_MAE_TOL and exact > 0.999
    assert segs == st.segments and lambs == st.lambertian


@pytest.mark.parametrize("robust", [0, 1])
def test_f32_sphere_test_forms_bvh_equals_brute(robust):
    """Both f32 ray-sphere forms (tuning "robust": the reference's hb^2 - a c,
    or the closest-approach form used for far geometry) give BVH == brute."""
    soa, b = _scene(11)
    cam = b.with_image_width(48).with_image_height(32).with_samples_per_pixel(4).with_max_depth(50).build()
    t = {"robust": robust, "light_bvh_min": 1 << 30}
    brute, _, cb = _render_gpu(soa, cam, 19, rtw.RTW_F32, accel=rtw.RTW_ACCEL_BRUTE, tuning=t)
    bvh, _, cv = _render_gpu(soa, cam, 19, rtw.RTW_F32, accel=rtw.RTW_ACCEL_BVH, tuning=t)
    assert _same(brute, bvh) and cb == cv


# ---- Quad + DiffuseLight

def _cornell_quads(with_metal=True):
    """scenes::cornell_box (scenes/src/lib.rs:292-395) without its rotated
    Cuboid (rank 4): the five walls, the ceiling light and the glass sphere;
    lights = [ceiling quad, glass sphere] in the reference's order."""
    red, white, green = rtw.Lambertian((0.65, 0.05, 0.05)), rtw.Lambertian((0.73, 0.73, 0.73)), \
        rtw.Lambertian((0.12, 0.45, 0.15))
    light, glass = rtw.DiffuseLight((15.0, 15.0, 15.0)), rtw.Dialectric(1.5)
    world = rtw.HittableList([
        rtw.Quad((555, 0, 0), (0, 555, 0), (0, 0, 555), green),
        rtw.Quad((0, 0, 0), (0, 555, 0), (0, 0, 555), red),
        rtw.Quad((0, 0, 0), (555, 0, 0), (0, 0, 555), white),
        rtw.Quad((555, 555, 555), (-555, 0, 0), (0, 0, -555), white),
        rtw.Quad((0, 0, 555), (555, 0, 0), (0, 555, 0), white),
        rtw.Quad((343, 554, 332), (-130, 0, 0), (0, 0, -105), light),
        rtw.Sphere((190, 90, 190), 90, glass),
    ])
    if with_metal:
        world.add(rtw.Sphere((400, 100, 350), 100, rtw.Metal((0.8, 0.85, 0.88), 0.05)))
    lights = rtw.HittableList([rtw.Quad((343, 554, 332), (-130, 0, 0), (0, 0, -105)),
                               rtw.Sphere((190, 90, 190), 90)])
    cam = rtw.CameraBuilder().with_lookfrom((278, 278, -800)).with_lookat((278, 278, 0)) \
        .with_vfov(40).with_background((0, 0, 0))
    return rtw.flatten(world, lights), cam


def test_quad_scene_f64_matches_oracle():
    soa, b = _cornell_quads()
    assert soa.light_kinds.tolist() == [1, 0]
    cam = b.with_image_width(40).with_image_height(40).with_samples_per_pixel(6).with_max_depth(30).build()
    for accel in (rtw.RTW_ACCEL_BRUTE, rtw.RTW_ACCEL_BVH):
        gpu, chunk, (segs, lambs) = _render_gpu(soa, cam, 61, rtw.RTW_F64, accel=accel)
        ref, st = _render_oracle(soa, cam, 61, chunk)
        mae, exact = _compare_f64(gpu, ref, 6)
        assert mae < F64_MAE_TOL and exact > 0.999, (accel, mae, exact)
        assert segs == st.segments and lambs == st.lambertian


def test_quad_scene_f32_bvh_equals_brute_and_tracks_f64():
    soa, b = _cornell_quads()
    cam = b.with_image_width(48).with_image_height(48).with_samples_per_pixel(16).with_max_depth(30).build()
    brute, _, cb = _render_gpu(soa, cam, 67, rtw.RTW_F32, accel=rtw.RTW_ACCEL_BRUTE)
    bvh, _, cv = _render_gpu(soa, cam, 67, rtw.RTW_F32, accel=rtw.RTW_ACCEL_BVH)
    assert _same(brute, bvh) and cb == cv
    ref, _ = _render_oracle(soa, cam, 67, 0)
    ok = ~(np.isnan(bvh).any(-1) | np.isnan(ref).any(-1))
    m32, m64 = bvh[ok].mean(), ref[ok].mean()
    assert abs(m32 - m64) < 0.03 * m64, (m32, m64)


def test_diffuse_light_quad_is_its_colour():
    world = rtw.HittableList([rtw.Quad((-5, -5, -3), (10, 0, 0), (0, 10, 0), rtw.DiffuseLight((4, 2, 1)))])
    soa = rtw.flatten(world, rtw.HittableList())
    cam = rtw.CameraBuilder().with_image_width(8).with_image_height(6).with_samples_per_pixel(5) \
        .with_max_depth(10).with_background((0, 0, 0)).build()
    for prec in (rtw.RTW_F32, rtw.RTW_F64):
        gpu, _, (segs, lambs) = _render_gpu(soa, cam, 3, prec)
        np.testing.assert_array_equal(gpu, np.broadcast_to([20.0, 10.0, 5.0], gpu.shape))
        assert segs == 8 * 6 * 5 and lambs == 0


def test_cornell_box_f64_matches_oracle():
    """scenes::cornell_box (scenes/src/lib.rs:292-395) in full: walls, light,
    glass sphere and the translated + rotated Cuboid (Transformed<Cuboid>
    with the reference's direction-translation behaviour).  The reference
    world is a flat HittableList (lib.rs:297, :392), so the oracle runs brute
    force: coplanar ties (floor vs the cuboid's bottom face) go to the first
    type group, as HittableList::hit's min_by does (hittable_list.rs:395-406)."""
    soa, b = rtw.scenes.cornell_box_soa()
    assert len(soa.box_mat) == 1 and soa.light_kinds.tolist() == [1, 0]
    cam = b.with_image_width(40).with_image_height(40).with_samples_per_pixel(4).with_max_depth(20).build()
    for accel in (rtw.RTW_ACCEL_BRUTE, rtw.RTW_ACCEL_BVH):
        gpu, chunk, (segs, lambs) = _render_gpu(soa, cam, 71, rtw.RTW_F64, accel=accel)
        ref, st = _render_oracle(soa, cam, 71, chunk, O.ACCEL_BRUTE)
        mae, exact = _compare_f64(gpu, ref, 4)
        assert mae < F64_MAE_TOL and exact > 0.999, (accel, mae, exact)
        assert segs == st.segments and lambs == st.lambertian


def test_cornell_box_f32_tracks_f64():
    soa, b = rtw.scenes.cornell_box_soa()
    cam = b.with_image_width(48).with_image_height(48).with_samples_per_pixel(32).with_max_depth(20).build()
    brute, _, cb = _render_gpu(soa, cam, 73, rtw.RTW_F32, accel=rtw.RTW_ACCEL_BRUTE)
    bvh, _, cv = _render_gpu(soa, cam, 73, rtw.RTW_F32, accel=rtw.RTW_ACCEL_BVH)
    assert _same(brute, bvh) and cb == cv
    ref, _ = _render_oracle(soa, cam, 73, 0, O.ACCEL_BRUTE)
    ok = ~(np.isnan(bvh).any(-1) | np.isnan(ref).any(-1))
    assert abs(bvh[ok].mean() - ref[ok].mean()) < 0.03 * ref[ok].mean()


# ---- textures, UVs and the remaining reference scenes

def _named(name, w, h, spp, depth, **over):
    soa, b = rtw.scenes.named_soa(name)
    b = b.with_image_width(w).with_image_height(h).with_samples_per_pixel(spp).with_max_depth(depth)
    for k, v in over.items():
        getattr(b, "with_" + k)(v)
    return soa, b.build()


@pytest.mark.parametrize("name", ["checkered_spheres", "simple_light", "debug", "simple_transform", "plane"])
@pytest.mark.parametrize("accel", [rtw.RTW_ACCEL_BRUTE, rtw.RTW_ACCEL_BVH])
def test_reference_scene_f64_matches_oracle(name, accel):
    """Every scenes/src/lib.rs generator with textures (checker on spheres,
    Perlin noise on planes and spheres), DiffuseLight spheres / quads /
    cuboids, BVH light lists and Hittable-default lights: the f64 kernel is
    bit-identical to the oracle (brute-force world, list tie order)."""
    soa, cam = _named(name, 32, 24, 4, 12, vfov=40.0)
    gpu, chunk, (segs, lambs) = _render_gpu(soa, cam, 83, rtw.RTW_F64, accel=accel)
    ref, st = _render_oracle(soa, cam, 83, chunk, O.ACCEL_BRUTE)
    mae, exact = _compare_f64(gpu, ref, 4)
    assert mae < F64_MAE_TOL and exact > 0.999, (name, mae, exact)
    assert segs == st.segments and lambs == st.lambertian


# integration-tests/src/lib.rs:7-112, each camera as the test builds it
INTEGRATION = {
    "plane_test": ("plane", dict(image_width=3, image_height=2, samples_per_pixel=10, max_depth=3,
                                 lookfrom=(-13, 2, 3), lookat=(0, 0, 0), vup=(0, 1, 0), focus_dist=10.0), True),
    "small_light_test": ("simple_light", dict(image_width=3, image_height=2, samples_per_pixel=10, max_depth=5,
                                              lookfrom=(4, 2, 10), lookat=(4, 2, -2), vup=(0, 1, 0),
                                              focus_dist=4.0), True),
    "debugging_test": ("debug", dict(image_width=3, image_height=2, samples_per_pixel=50, max_depth=10,
                                     vfov=40.0, lookat=(0, 0, 0), lookfrom=(0, 20, 0)), False),
    "cornell_box_test": ("cornell_box", dict(image_width=3, image_height=2, samples_per_pixel=50,
                                             max_depth=10, vfov=40.0), False),
}


@pytest.mark.parametrize("test", sorted(INTEGRATION))
def test_integration_test_configs_f64_match_oracle(test):
    """The reference's own smoke renders (integration-tests/src/lib.rs) --
    which assert only 'does not panic' -- rendered through the C-ABI and
    compared bit for bit with the oracle."""
    name, kw, fresh = INTEGRATION[test]
    soa, b = rtw.scenes.named_soa(name)
    if fresh:
        b = rtw.CameraBuilder()
    for k, v in kw.items():
        getattr(b, "with_" + k)(v)
    cam = b.build()
    gpu, chunk, (segs, lambs) = _render_gpu(soa, cam, 89, rtw.RTW_F64)
    ref, st = _render_oracle(soa, cam, 89, chunk, O.ACCEL_BRUTE)
    mae, exact = _compare_f64(gpu, ref, cam.raw.samples_per_pixel)
    assert mae < F64_MAE_TOL and exact == 1.0 and segs == st.segments


def test_perlin_spheres_panics_like_the_reference():
    """perlin_spheres (scenes/src/lib.rs:40-89) has no lights: the reference
    panics on the first Lambertian light draw; the C-ABI returns
    RTW_E_NO_LIGHTS and counts the same draws as the oracle."""
    soa, cam = _named("perlin_spheres", 16, 16, 2, 10)
    ref, st = _render_oracle_allow_panic(soa, cam, 97, 1)
    with rtw.Renderer(precision=rtw.RTW_F64) as r:
        r.set_scene(soa)
        with pytest.raises(rtw.RenderError) as e:
            r.render(cam, 97)
        assert e.value.code == -3 and r.stats.panic_no_lights == st.panic_no_lights > 0


def test_down_facing_plane_panics_like_the_reference():
    """Plane::hit computes the UV before its range test; for n = -y it is NaN
    and the reference panics (plane.rs:66-69): RTW_E_PANIC, same count."""
    world = rtw.HittableList([rtw.Plane((0, -1, 0), (0, -1, 0), rtw.Lambertian((0.5, 0.5, 0.5))),
                              rtw.Sphere((0, 0, -2), 0.5, rtw.Metal((0.8, 0.8, 0.8), 0.0))])
    soa = rtw.flatten(world, rtw.HittableList([rtw.Sphere((0, 5, 0), 1.0)]))
    cam = rtw.CameraBuilder().with_image_width(8).with_image_height(8).with_samples_per_pixel(2) \
        .with_lookfrom((0, 3, 0)).with_lookat((0, 0, 0.1)).build()
    ref, st = _render_oracle_allow_panic(soa, cam, 3, 1)
    assert st.panic_plane_uv > 0
    with rtw.Renderer(precision=rtw.RTW_F64) as r:
        r.set_scene(soa)
        with pytest.raises(rtw.RenderError) as e:
            r.render(cam, 3)
        assert e.value.code == -6 and r.stats.panic_plane_uv == st.panic_plane_uv


@pytest.mark.parametrize("name", ["checkered_spheres", "simple_light", "debug"])
def test_reference_scene_f32_tracks_f64(name):
    """f32 speed mode on the textured scenes: BVH == brute force bit for bit,
    image mean within 3 % of the f64 oracle."""
    soa, cam = _named(name, 48, 32, 16, 12, vfov=40.0)
    brute, _, cb = _render_gpu(soa, cam, 101, rtw.RTW_F32, accel=rtw.RTW_ACCEL_BRUTE)
    bvh, _, cv = _render_gpu(soa, cam, 101, rtw.RTW_F32, accel=rtw.RTW_ACCEL_BVH)
    assert _same(brute, bvh) and cb == cv
    ref, _ = _render_oracle(soa, cam, 101, 0, O.ACCEL_BRUTE)
    ok = ~(np.isnan(bvh).any(-1) | np.isnan(ref).any(-1))
    assert abs(bvh[ok].mean() - ref[ok].mean()) < 0.03 * ref[ok].mean(), (bvh[ok].mean(), ref[ok].mean())


def test_python_textured_scene_on_the_gpu():
    """The Python mirror's textures (CheckerTexture of a NoiseTexture, a
    textured DiffuseLight) through flatten and the C-ABI, vs the oracle."""
    noise = rtw.NoiseTexture.new(2.0, 7)
    check = rtw.CheckerTexture.new(noise, rtw.SolidColour((0.9, 0.2, 0.1)), 0.5)
    world = rtw.HittableList([
        rtw.Sphere((0, 0, -2), 1.0, rtw.Lambertian(check)),
        rtw.Quad((-3, -1, -5), (6, 0, 0), (0, 4, 0), rtw.Lambertian(rtw.CheckerTexture.new_with_colours(
            (0.1, 0.1, 0.1), (0.8, 0.8, 0.8), 0.1))),
        rtw.Sphere((1.5, 1.2, -1.5), 0.3, rtw.DiffuseLight(rtw.CheckerTexture.new_with_colours(
            (4, 4, 4), (1, 0, 0), 0.05))),
        rtw.Plane((0, -1, 0), (0, 1, 0.2), rtw.Lambertian(noise)),
    ])
    lights = rtw.HittableList([rtw.Sphere((1.5, 1.2, -1.5), 0.3)])
    soa = rtw.flatten(world, lights)
    cam = rtw.CameraBuilder().with_image_width(32).with_image_height(24).with_samples_per_pixel(4) \
        .with_max_depth(12).with_lookfrom((0, 0.5, 2)).with_lookat((0, 0, -2)).with_vfov(60) \
        .with_background((0.2, 0.3, 0.4)).build()
    gpu, chunk, _ = _render_gpu(soa, cam, 103, rtw.RTW_F64)
    ref, _ = _render_oracle(soa, cam, 103, chunk, O.ACCEL_BRUTE)
    mae, exact = _compare_f64(gpu, ref, 4)
    assert mae < F64_MAE_TOL and exact > 0.999


# ---- BASELINE.json's headline size (C2: 1200 x 800, depth 50) at few spp:
# every 40th row against the oracle, and the rank split reassembled

def test_c2_full_frame_f64_rows_match_oracle():
    soa, b = _scene()
    cam = b.with_image_width(1200).with_image_height(800).with_samples_per_pixel(3).with_max_depth(50).build()
    gpu, chunk, _ = _render_gpu(soa, cam, 107, rtw.RTW_F64)
    ocam = O.Camera()
    for name, _ in O.Camera._fields_:
        setattr(ocam, name, getattr(cam.raw, name))
    ref, st = O.render(ocam, O.Scene(**soa.__dict__), 107, chunk=chunk, accel=O.ACCEL_BVH_CACHED,
                       rows=(3, 800, 40))
    rows = list(range(3, 800, 40))
    mae, exact = _compare_f64(gpu[rows], ref[rows], 3)
    assert mae < F64_MAE_TOL and exact == 1.0, (mae, exact)


@pytest.mark.parametrize("nranks,lpt", [(2, 0), (8, 0), (3, 1), (8, 1)])
def test_c2_full_frame_rank_split_is_the_single_render(nranks, lpt):
    """rtw_render_device over nranks (the multi-GPU tile interleave, DESIGN.md
    §7) + rtw_assemble_tiles reassembles the one-rank C2-size image bit for
    bit (f32).  Every render runs on torch's current stream, the stream the
    buffers were filled on.  lpt: each rank's share and then the one-rank
    frame again are rendered twice, the second time with its tiles longest
    first, in the order of the tile costs the first render counted."""
    import torch
    soa, b = _scene()
    H, W = 800, 1200
    cam = b.with_image_width(W).with_image_height(H).with_samples_per_pixel(2).with_max_depth(50).build()
    s = rtw.torch_stream(torch.cuda.current_device())
    with rtw.Renderer(precision=rtw.RTW_F32) as r:
        r.set_tuning("lpt", lpt)
        r.set_tuning("lpt_min_spp", 1)
        r.set_scene(soa)
        one = torch.zeros((rtw.tiles_for_rank(W, H, 0, 1) * 64 * 3,), dtype=torch.float32, device="cuda:0")
        r.render_device(cam, 109, one.data_ptr(), one.numel() * 4, stream=s)
        full = torch.zeros((H, W, 3), dtype=torch.float32, device="cuda:0")
        r.assemble_tiles(one.data_ptr(), one.numel() * 4, 1, W, H, full.data_ptr(), stream=s)
        per = rtw.tiles_for_rank(W, H, 0, nranks) * 64 * 3
        ranks = torch.zeros((nranks, per), dtype=torch.float32, device="cuda:0")
        for k in range(nranks):
            for _ in range(1 + lpt):   # lpt: the second render of a share takes its ordered task list
                r.render_device(cam, 109, ranks[k].data_ptr(), per * 4, rank=k, nranks=nranks, stream=s)
        img = torch.empty_like(full)
        r.assemble_tiles(ranks.data_ptr(), per * 4, nranks, W, H, img.data_ptr(), stream=s)
        again = torch.zeros_like(one)
        for _ in range(1 + lpt):
            r.render_device(cam, 109, again.data_ptr(), again.numel() * 4, stream=s)
        torch.cuda.synchronize()
    assert torch.equal(torch.nan_to_num(img, nan=-7.0), torch.nan_to_num(full, nan=-7.0))
    assert torch.equal(torch.nan_to_num(again, nan=-7.0), torch.nan_to_num(one, nan=-7.0))


@pytest.mark.parametrize("prec", [rtw.RTW_F32, rtw.RTW_F64])
def test_scheduling_knobs_do_not_change_the_image(prec):
    """The wave item pool order (pixel- / sample-major), persistent waves (a
    few workgroups draining every task from the counter, or a resident grid) or
    one task per wave and the task size only move work between lanes, and the
    longest-tiles-first task order (the tile costs the first render counts,
    or a separate pilot render's) only moves tiles between tasks: same image
    bit for bit."""
    soa, b = _scene()
    cam = b.with_image_width(40).with_image_height(24).with_samples_per_pixel(9).with_max_depth(50).build()
    base, _, cb = _render_gpu(soa, cam, 113, prec)
    for t in ({"item_order": 0}, {"persist": 2}, {"persist": 3, "group": 1}, {"persist": 0},
              {"persist": 0, "target_tasks": 1000}, {"item_order": 0, "target_tasks": 1000},
              {"persist": 5, "group": 3}, {"persist": 1, "group": 2},
              {"lpt_min_spp": 1}, {"lpt_min_spp": 1, "persist": 0}, {"lpt_min_spp": 1, "persist": 2, "group": 1},
              {"lpt": 2, "lpt_min_spp": 1, "lds": 0}, {"lpt_min_spp": 1, "lpt_inline": 0},
              {"lpt_min_spp": 1, "lpt_inline": 0, "lpt_pilot_depth": 3}):
        img, _, cv = _render_gpu(soa, cam, 113, prec, tuning=t, renders=3 if "lpt_min_spp" in t else 1)
        assert _same(base, img) and cb == cv, t


def test_task_table_with_4096_chunk_groups_keeps_every_chunk():
    """A fixed group of 4096 chunks at chunk 1 with the task table on: the
    table entry holds the chunk count in 12 bits, so the host cuts such tasks
    at 4095 chunks (a 4096 would wrap to 0 and the kernel would skip the
    task, leaving its chunk sums unwritten).  Same image bit for bit as the
    plain tile-major schedule."""
    soa, b = _scene()
    cam = b.with_image_width(16).with_image_height(8).with_samples_per_pixel(4100).with_max_depth(6).build()
    base, chunk, cb = _render_gpu(soa, cam, 131, rtw.RTW_F32, tuning={"lpt": 0})
    assert chunk == 1
    img, _, cv = _render_gpu(soa, cam, 131, rtw.RTW_F32,
                             tuning={"group": 4096, "lpt_min_spp": 1, "chunk": 1}, renders=2)
    assert _same(base, img) and cb == cv


@pytest.mark.parametrize("kind", [0, 2, 3])
def test_textured_light_grid_scene_every_bvh_kind(kind):
    """an f64 textured scene whose light list takes the light grid
    (>= 64 sphere lights) renders under every BVH kind -- the textured kernels'
    per-lane grid walk needs no stash or piece slots, so the remapped binary
    kernels must not ask for them -- bit-identical to the oracle."""
    soa, b = _scene(20)
    assert np.asarray(soa.lights).reshape(-1, 4).shape[0] >= 64
    nm = len(soa.mat_type)
    soa.tex_type = np.array([rtw.RTW_TEX_SOLID] * (nm + 2) + [rtw.RTW_TEX_CHECKER], np.uint32)
    soa.tex_params = np.array([list(soa.mat_params[m][:3]) + [0.0] for m in range(nm)] +
                              [[0.2, 0.3, 0.1, 0.0], [0.9, 0.9, 0.9, 0.0], [0.0, 0.0, 0.0, 1.0 / 0.32]], np.float64)
    soa.tex_refs = np.array([[0, 0]] * (nm + 2) + [[nm, nm + 1]], np.uint32)
    mat_tex = np.arange(nm, dtype=np.uint32)
    mat_tex[soa.plane_mat[0]] = nm + 2                      # the ground: a checker
    soa.mat_tex = mat_tex
    cam = b.with_image_width(40).with_image_height(24).with_samples_per_pixel(4).with_max_depth(50).build()
    # (textured scenes run the binary while-while kernel for kinds 0 and 2)
    gpu, chunk, (segs, lambs) = _render_gpu(soa, cam, 5, rtw.RTW_F64, accel=rtw.RTW_ACCEL_BVH,
                                            tuning={"bvh_kind": kind, "bvh_lds_max": 64 * 1024})
    assert LAST["kernel"] in (K_BVH_WW, K_BVH_LDS)
    ref, st = _render_oracle(soa, cam, 5, chunk)
    mae, exact = _compare_f64(gpu, ref, 4)
    assert mae < F64_MAE_TOL and exact > 0.999
    assert segs == st.segments and lambs == st.lambertian
