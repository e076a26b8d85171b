"""The multi-device context of the C-ABI (ABI 8: rtw_create_devices /
rtw_create_mask, SURVEY.md §8(b)(1)'s device_mask): every GPU of the context
renders its 8x8 tiles (T = rank mod n), one RCCL gather (ncclGather from a
single-process ncclCommInitAll clique) brings them to the first GPU, which
assembles the image.  On a one-GPU box the context has one rank, which still
runs the whole path (RCCL clique, gather, assembly); with two or more GPUs
visible the n-rank image is checked too.  The image must be bit-identical to
a plain one-GPU rtw_render of the same seed."""
import ctypes as C

import numpy as np
import pytest
import torch

import ray_tracing_weekend_amd as rtw

pytestmark = pytest.mark.gpu

SEED = 0x5EED0001


def _cam(w=72, h=40, spp=6):
    scene, b = rtw.scenes.simple_soa(SEED)
    return scene, b.with_image_width(w).with_image_height(h).with_samples_per_pixel(spp).with_max_depth(50).build()


def _single(scene, cam, prec, seed=11):
    with rtw.Renderer(device=0, precision=prec) as r:
        r.set_scene(scene)
        img = r.render(cam, seed)
        return img, r.stats.samples, r.stats.segments


@pytest.mark.parametrize("prec", [rtw.RTW_F64, rtw.RTW_F32])
def test_one_device_context_is_bit_identical_to_rtw_render(prec):
    scene, cam = _cam()
    ref, samples, segments = _single(scene, cam, prec)
    with rtw.Renderer(precision=prec, devices=[0]) as r:
        assert r.n_devices == 1
        r.set_scene(scene)
        img = r.render(cam, 11)
        assert r.stats.samples == samples == cam.image_width * cam.image_height * cam.samples_per_pixel
        assert r.stats.segments == segments
    assert np.array_equal(np.isnan(img), np.isnan(ref))
    ok = ~np.isnan(ref)
    assert np.array_equal(img[ok], ref[ok])


def test_mask_context_and_image_device_match():
    """rtw_create_mask(1) (device 0) and rtw_render_image_device into a torch
    tensor on torch's stream: the same image as rtw_render."""
    scene, cam = _cam(w=37, h=23, spp=5)      # ragged tiles
    ref, _, _ = _single(scene, cam, rtw.RTW_F64, seed=3)
    ctx = rtw._lib.rtw_create_mask(1, rtw.RTW_F64)
    assert ctx
    try:
        assert rtw._lib.rtw_device_count(ctx) == 1
        assert rtw._lib.rtw_device_of(rtw._lib.rtw_device_ctx(ctx, 0)) == 0
        assert rtw._lib.rtw_device_ctx(ctx, 1) is None
        s, keep = scene.as_c()
        assert rtw._lib.rtw_set_scene(ctx, C.byref(s)) == 0
        img = torch.full((cam.image_height, cam.image_width, 3), float("nan"), dtype=torch.float64, device="cuda:0")
        stream = rtw.torch_stream(0)
        rc = rtw._lib.rtw_render_image_device(ctx, C.byref(cam.raw), C.c_uint64(3), C.c_void_p(img.data_ptr()),
                                              img.numel() * 8, C.c_void_p(stream))
        assert rc == 0, rtw._lib.rtw_last_error(ctx)
        got = img.cpu().numpy()
        # a too-small image buffer is refused, not overrun
        assert rtw._lib.rtw_render_image_device(ctx, C.byref(cam.raw), C.c_uint64(3), C.c_void_p(img.data_ptr()),
                                                img.numel() * 8 - 8, C.c_void_p(stream)) == rtw._capi.RTW_E_INVALID
    finally:
        rtw._lib.rtw_destroy(ctx)
    ok = ~np.isnan(ref)
    assert np.array_equal(np.isnan(got), np.isnan(ref)) and np.array_equal(got[ok], ref[ok])


def test_repeated_device_rejected():
    with pytest.raises(rtw.RenderError) as e:
        rtw.Renderer(precision=rtw.RTW_F64, devices=[0, 0])
    assert e.value.code == rtw._capi.RTW_E_INVALID
    n = torch.cuda.device_count()
    with pytest.raises(rtw.RenderError):
        rtw.Renderer(precision=rtw.RTW_F64, devices=[0, n])      # not visible


def test_knobs_and_rank_views_follow_every_rank():
    scene, cam = _cam(w=64, h=64, spp=40)
    with rtw.Renderer(precision=rtw.RTW_F32, devices=list(range(torch.cuda.device_count()))) as r:
        r.set_tuning("lpt_min_spp", 8)
        r.set_scene(scene)
        a = r.render(cam, 5)
        b = r.render(cam, 5)          # second render: the task list of the counted costs (lpt)
        assert np.array_equal(np.nan_to_num(a, nan=-1), np.nan_to_num(b, nan=-1))
        tot = 0
        for k in range(r.n_devices):
            v = r.rank_view(k)
            st = v.get_stats()
            tot += st.samples
            assert v.last_kernel() is not None and len(v.get_timings(2)[0]) == 2
        assert tot == r.stats.samples == 64 * 64 * 40


@pytest.mark.skipif(torch.cuda.device_count() < 2, reason="needs two GPUs")
@pytest.mark.parametrize("prec", [rtw.RTW_F64, rtw.RTW_F32])
def test_n_device_context_is_bit_identical(prec):
    scene, cam = _cam(w=120, h=72, spp=4)
    ref, samples, _ = _single(scene, cam, prec, seed=9)
    n = torch.cuda.device_count()
    with rtw.Renderer(precision=prec, devices=list(range(n))) as r:
        r.set_tuning("lpt_min_spp", 2)
        r.set_scene(scene)
        img = r.render(cam, 9)                   # counting render (the round robin)
        assert r.stats.samples == samples
        dealt = r.render(cam, 9)                 # the tiles dealt by their costs (ABI 10)
        assert r.stats.samples == samples
    ok = ~np.isnan(ref)
    for a in (img, dealt):
        assert np.array_equal(np.isnan(a), np.isnan(ref)) and np.array_equal(a[ok], ref[ok])


# ---- the n-rank path on one GPU: rtw_create_virtual (ABI 9, test mode) ------
# Every rank of the context lives on device 0 and the gather is device copies
# on rank 0's stream; everything else is the product path (per-rank contexts,
# streams, buffers and scene copies, rank 0 rendering into its gather slot,
# the assembly, the summed stats, the per-rank longest-first task lists).


@pytest.mark.parametrize("prec", [rtw.RTW_F64, rtw.RTW_F32])
@pytest.mark.parametrize("n", [2, 3, 8])
def test_virtual_ranks_bit_identical(prec, n):
    scene, cam = _cam(w=120, h=72, spp=40)          # 15 x 9 tiles: ragged over 2, 3 and 8 ranks
    with rtw.Renderer(device=0, precision=prec) as r:
        r.set_tuning("lpt_min_spp", 8)
        r.set_scene(scene)
        ref = r.render(cam, 9)
        st = r.stats
        ref_samples, ref_segments, ref_lamb = st.samples, st.segments, st.lambertian
    with rtw.Renderer(device=0, precision=prec, virtual_ranks=n) as r:
        assert r.n_devices == n
        r.set_tuning("lpt_min_spp", 8)
        r.set_scene(scene)
        a = r.render(cam, 9)                         # counting render (tile index order)
        assert r.stats.samples == ref_samples == cam.image_width * cam.image_height * cam.samples_per_pixel
        assert r.stats.segments == ref_segments and r.stats.lambertian == ref_lamb
        assert r.stats.light_tests == ref_lamb * np.asarray(scene.lights).reshape(-1, 4).shape[0]
        b = r.render(cam, 9)                         # every rank's longest-first task list
        assert r.stats.segments == ref_segments
        per_rank = sum(r.rank_view(k).get_stats().samples for k in range(n))
        assert per_rank == ref_samples
    ok = ~np.isnan(ref)
    for img in (a, b):
        assert np.array_equal(np.isnan(img), np.isnan(ref)) and np.array_equal(img[ok], ref[ok])


@pytest.mark.parametrize("prec", [rtw.RTW_F64, rtw.RTW_F32])
def test_virtual_ranks_image_device_streams_and_stats(prec):
    """rtw_render_image_device of a virtual 3-rank context on two different
    torch streams back to back (the second call's renders wait for the first
    call's gather + assembly), then rtw_render_device on the same context:
    its stats are rank 0's alone.  (The RCCL transport's cross-device event
    wait has the same order but runs only on >= 2 GPUs.)"""
    scene, cam = _cam(w=64, h=48, spp=6)
    ref, samples, _ = _single(scene, cam, prec, seed=4)
    tdt = torch.float64 if prec == rtw.RTW_F64 else torch.float32
    with rtw.Renderer(device=0, precision=prec, virtual_ranks=3) as r:
        r.set_scene(scene)
        imgs = []
        for k in range(2):
            s = torch.cuda.Stream()
            with torch.cuda.stream(s):
                img = torch.full((cam.image_height, cam.image_width, 3), float("nan"), dtype=tdt,
                                 device="cuda:0")
                r.render_image_device(cam, 4, img.data_ptr(), img.numel() * img.element_size())
                imgs.append(img.cpu().double().numpy())
        assert r.get_stats().samples == samples
        n0 = rtw.tiles_for_rank(cam.image_width, cam.image_height, 0, 1) * 64 * 3
        out = torch.zeros(n0, dtype=tdt, device="cuda:0")
        r.render_device(cam, 4, out.data_ptr(), out.numel() * out.element_size())
        torch.cuda.synchronize()
        assert r.get_stats().samples == samples      # one rank rendered everything: rank 0's stats
        v = r.rank_view(1)
    with pytest.raises(rtw.RenderError):
        v.get_stats()                                # the parent is closed
    ok = ~np.isnan(ref)
    for got in imgs:
        assert np.array_equal(np.isnan(got), np.isnan(ref)) and np.array_equal(got[ok], ref[ok])


def test_virtual_ranks_light_grid_counters():
    """A scene whose light pdf takes the light grid (>= 64 lights): the image
    and the segments of a 3-rank render equal the one-rank render's.  The
    light tests and grid cells (ABI 9) are WALK-WORK counters of the
    cooperative walks -- a boundary cell is visited by both adjacent pieces,
    the piece length adapts to the wave's pending cells, a re-walk counts its
    cells again -- so they depend on how rays are grouped into waves: the
    3-rank sums agree with the one-rank counts within a few percent, not bit
    for bit."""
    scene, b = rtw.scenes.simple_soa(SEED, n=20)
    cam = b.with_image_width(48).with_image_height(32).with_samples_per_pixel(4).with_max_depth(50).build()
    assert np.asarray(scene.lights).reshape(-1, 4).shape[0] >= 64
    with rtw.Renderer(device=0, precision=rtw.RTW_F64) as r:
        r.set_scene(scene)
        ref = r.render(cam, 2)
        st = (r.stats.light_tests, r.stats.grid_cells, r.stats.segments)
        assert r.last_kernel()[1] & 2                # the light grid / BVH kernel ran
    assert st[0] > 0 and st[1] > 0
    with rtw.Renderer(device=0, precision=rtw.RTW_F64, virtual_ranks=3) as r:
        r.set_scene(scene)
        img = r.render(cam, 2)
        assert r.stats.segments == st[2]
        assert abs(r.stats.light_tests / st[0] - 1) < 0.05 and abs(r.stats.grid_cells / st[1] - 1) < 0.05
    ok = ~np.isnan(ref)
    assert np.array_equal(np.isnan(img), np.isnan(ref)) and np.array_equal(img[ok], ref[ok])


# ---- the cost-dealt rank split (ABI 10) ------------------------------------


@pytest.mark.parametrize("prec", [rtw.RTW_F64, rtw.RTW_F32])
@pytest.mark.parametrize("n", [2, 3, 8])
def test_virtual_ranks_balance_deals_by_cost_bit_identical(prec, n):
    """A multi-device context deals its tiles by their counted costs by
    itself (tuning "balance"): the first render of the camera counts (round
    robin), the second deals (rtw_get_split kind 2, each rank keeping its
    round-robin tile count) and renders balanced; every image bit-identical
    to a one-rank render, the summed counters too."""
    scene, cam = _cam(w=120, h=72, spp=40)
    W, H = cam.image_width, cam.image_height
    with rtw.Renderer(device=0, precision=prec) as r:
        r.set_tuning("lpt_min_spp", 8)
        r.set_scene(scene)
        ref = r.render(cam, 9)
        ref_segments = r.stats.segments
    ok = ~np.isnan(ref)
    with rtw.Renderer(device=0, precision=prec, virtual_ranks=n) as r:
        r.set_tuning("lpt_min_spp", 8)
        r.set_scene(scene)
        imgs = [r.render(cam, 9)]
        assert r.get_split(W, H, n)[0] == 0                 # counted under the round robin
        imgs.append(r.render(cam, 9))
        kind, split = r.get_split(W, H, n)
        assert kind == 2
        assert np.bincount(split, minlength=n).tolist() == [rtw.tiles_for_rank(W, H, k, n) for k in range(n)]
        rr = np.arange(split.size) % n
        assert not np.array_equal(split, rr)
        assert r.stats.segments == ref_segments
        assert sum(r.rank_view(k).get_stats().samples for k in range(n)) == W * H * cam.samples_per_pixel
        imgs.append(r.render(cam, 9))                       # steady state on the dealt split
        for k in range(n):                                  # every rank holds the same split
            assert np.array_equal(r.rank_view(k).get_split(W, H, n)[1], split)
    for img in imgs:
        assert np.array_equal(np.isnan(img), np.isnan(ref)) and np.array_equal(img[ok], ref[ok])


def test_virtual_ranks_balance_off_keeps_round_robin():
    scene, cam = _cam(w=64, h=48, spp=40)
    with rtw.Renderer(device=0, precision=rtw.RTW_F64, virtual_ranks=2) as r:
        r.set_tuning("lpt_min_spp", 8)
        r.set_tuning("balance", 0)
        r.set_scene(scene)
        r.render(cam, 1)
        r.render(cam, 1)
        assert r.get_split(cam.image_width, cam.image_height, 2)[0] == 0


@pytest.mark.parametrize("prec", [rtw.RTW_F64, rtw.RTW_F32])
def test_explicit_split_render_device_and_assemble(prec):
    """rtw_set_split + rtw_render_device(rank, n) + rtw_assemble_tiles on one
    context: each rank's packed buffer holds exactly its dealt tiles in
    increasing tile order (sharding.pack with the split), the assembled
    image equals a plain render bit for bit; tile costs from the counting
    render of each rank cover exactly its tiles."""
    from ray_tracing_weekend_amd import sharding
    scene, cam = _cam(w=77, h=45, spp=33)             # ragged tiles
    W, H, n = cam.image_width, cam.image_height, 3
    tdt = torch.float64 if prec == rtw.RTW_F64 else torch.float32
    with rtw.Renderer(device=0, precision=prec) as r:
        r.set_scene(scene)
        ref = r.render(cam, 5)
        per = rtw.tiles_for_rank(W, H, 0, n) * 64 * 3
        bufs = torch.full((n, per), float("nan"), dtype=tdt, device="cuda:0")
        with pytest.raises(rtw.RenderError):
            r.tile_costs(cam, 0, n)                         # nothing counted for this split yet
        costs = np.zeros(rtw.n_tiles(W, H), np.uint32)
        r.set_tuning("lpt_min_spp", 8)
        for k in range(n):                                  # counting renders (round robin)
            r.render_device(cam, 5, bufs[k].data_ptr(), per * bufs.element_size(), rank=k, nranks=n)
            before = costs.copy()
            r.tile_costs(cam, k, n, out=costs)
            changed = np.nonzero(costs != before)[0]
            assert set(changed.tolist()) <= set(sharding.rank_tiles(W, H, k, n))
        assert (costs > 0).mean() > 0.9
        split = rtw.split_deal(costs, W, H, n)
        bad = split.copy()
        bad[0] = (bad[0] + 1) % n                           # one rank a tile too many
        with pytest.raises(rtw.RenderError):
            r.set_split(W, H, n, bad)
        r.set_split(W, H, n, split, costs)
        assert r.get_split(W, H, n)[0] == 1
        assert r.get_split(W, H, n + 1)[0] == 0             # other rank counts: the round robin
        for k in range(n):
            r.render_device(cam, 5, bufs[k].data_ptr(), per * bufs.element_size(), rank=k, nranks=n)
        img = torch.empty((H, W, 3), dtype=tdt, device="cuda:0")
        r.assemble_tiles(bufs.data_ptr(), bufs.stride(0) * bufs.element_size(), n, W, H, img.data_ptr())
        torch.cuda.synchronize()
        got = img.cpu().double().numpy()
        full = torch.from_numpy(ref.astype(np.float32 if prec == rtw.RTW_F32 else np.float64))
        for k in range(n):
            p = sharding.pack(full, k, n, split).reshape(-1)
            b = bufs[k].cpu()[: p.numel()]
            assert torch.equal(torch.nan_to_num(b, nan=-1.0), torch.nan_to_num(p.to(b.dtype), nan=-1.0))
        r.set_split(W, H, n, None)                          # back to the round robin
        assert r.get_split(W, H, n)[0] == 0
    ok = ~np.isnan(ref)
    assert np.array_equal(np.isnan(got), np.isnan(ref)) and np.array_equal(got[ok], ref[ok])
