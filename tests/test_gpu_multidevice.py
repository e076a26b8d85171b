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
        r.set_scene(scene)
        img = r.render(cam, 9)
        assert r.stats.samples == samples
    ok = ~np.isnan(ref)
    assert np.array_equal(np.isnan(img), np.isnan(ref)) and np.array_equal(img[ok], ref[ok])
