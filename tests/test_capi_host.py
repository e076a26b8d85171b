"""CPU-side tests of the product: the C-ABI library loads and exports every
symbol include/rtw.h declares; the C++ host mirror (CameraBuilder::build,
scenes::simple, output encoding) agrees with the oracle restatement; nothing
here launches a kernel."""
import ctypes as C
import os
import math
import re

import numpy as np
import pytest

import ray_tracing_weekend_amd as rtw
from ray_tracing_weekend_amd import _capi
from oracle import oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared_symbols():
    text = open(os.path.join(ROOT, "include", "rtw.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(rtw_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    lib = C.CDLL(_capi.LIB_PATH)
    names = _declared_symbols()
    assert len(names) >= 20
    for n in names:
        assert hasattr(lib, n), n
    assert {p[0] for p in _capi.PROTOTYPES} == set(names)


def test_abi_version():
    assert rtw._lib.rtw_abi_version() == rtw._capi.ABI_VERSION == 10


def test_camera_builder_defaults_match_reference():
    b = rtw.CameraBuilder().raw           # camera.rs:45-60
    assert (b.samples_per_pixel, b.max_depth, b.vfov, b.focus_dist, b.defocus_angle) == (10, 10, 90.0, 10.0, 0.0)
    assert list(b.lookat) == [0.0, 0.0, -1.0] and list(b.vup) == [0.0, 1.0, 0.0]
    assert not (b.has_aspect_ratio or b.has_image_width or b.has_image_height)


@pytest.mark.parametrize("kw", [
    {},                                                    # (None, None, None) -> 100x100
    {"image_width": 64},
    {"image_height": 50},
    {"aspect_ratio": 16 / 9},
    {"image_width": 400, "image_height": 225},
    {"aspect_ratio": 1.5, "image_width": 301},
    {"aspect_ratio": 1.5, "image_height": 99},
    {"aspect_ratio": 2.0, "image_width": 10, "image_height": 3},
    {"lookfrom": (0, 5, 0), "lookat": (0, 0, 0)},         # vup x w ~ 0: the +0.1x nudge
    {"defocus_angle": 0.6, "focus_dist": 3.4, "vfov": 20.0},
])
def test_camera_build_matches_oracle(kw):
    b = rtw.CameraBuilder()
    for k, v in kw.items():
        getattr(b, "with_" + k)(v)
    cam = b.build()
    ocam = O.camera_build(**kw)
    for name, _ in O.Camera._fields_:
        a, c = getattr(cam.raw, name), getattr(ocam, name)
        a = list(a) if isinstance(a, C.Array) else a
        c = list(c) if isinstance(c, C.Array) else c
        assert a == c, name


def test_camera_known_answer_simple():
    """Analytic pixel00 for scenes::simple's camera (camera.rs:161-188)."""
    _, b = rtw.scenes.simple_soa()
    cam = b.with_image_width(400).with_image_height(225).build()
    lookfrom = np.array([10.0, 5.0, 10.0])
    f = np.linalg.norm(lookfrom)
    w = lookfrom / f
    u = np.cross([0, 1, 0], w)
    u /= np.linalg.norm(u)
    v = np.cross(w, u)
    vh = 2 * np.tan(np.radians(40) / 2) * f
    vw = vh * 400 / 225
    p00 = lookfrom - w * f - u * vw / 2 - v * vh / 2 + (u * vw / 400 + v * vh / 225) / 2
    np.testing.assert_allclose(cam.pixel00_loc, p00, rtol=0, atol=1e-12)
    np.testing.assert_allclose(cam.pixel_delta_u, u * vw / 400, atol=1e-14)
    np.testing.assert_allclose(cam.pixel_delta_v, v * vh / 225, atol=1e-14)
    assert cam.pixel_delta_v[1] > 0       # j = 0 is the bottom row


@pytest.mark.parametrize("seed,n", [(0x5EED0001, 11), (1, 11), (42, 3), (7, 0), (0xFFFFFFFFFFFFFFFF, 2)])
def test_scene_simple_matches_oracle(seed, n):
    soa, _ = rtw.scenes.simple_soa(seed, n)
    osc = O.scene_simple(seed, n)
    for f in ("spheres", "sphere_mat", "planes", "plane_mat", "mat_type", "mat_params", "lights"):
        np.testing.assert_array_equal(getattr(soa, f), getattr(osc, f), err_msg=f)


def test_scene_simple_structure():
    """scenes/src/lib.rs:155-233: 1 ground plane, <= 484 small + 3 big spheres,
    one light per glass sphere, materials drawn from the stated ranges."""
    soa, b = rtw.scenes.simple_soa(0x5EED0001)
    assert len(soa.plane_mat) == 1 and list(soa.planes[0]) == [0, 0, 0, 0, 1, 0]
    small = soa.spheres[:-3]
    assert np.all(small[:, 1] == 0.2) and np.all(small[:, 3] == 0.2)
    assert np.all(np.linalg.norm(small[:, :3] - [4, 0.2, 0], axis=1) > 0.9)
    np.testing.assert_array_equal(soa.spheres[-3:], [[0, 1, 0, 1], [-4, 1, 0, 1], [4, 1, 0, 1]])
    glass = soa.mat_type[soa.sphere_mat] == rtw.RTW_DIELECTRIC
    assert glass.sum() == len(soa.lights)
    mt, mp = soa.mat_type, soa.mat_params
    metal = mp[mt == rtw.RTW_METAL]
    assert np.all((metal[:, :3] >= 0.5) & (metal[:, :3] <= 1.0)) and np.all((metal[:, 3] >= 0) & (metal[:, 3] <= 0.5))
    lamb = mp[mt == rtw.RTW_LAMBERTIAN]
    assert np.all((lamb[:, :3] >= 0) & (lamb[:, :3] < 1))
    assert b.raw.vfov == 40.0 and list(b.raw.background) == [1, 1, 1]
    assert b.raw.focus_dist == pytest.approx(np.sqrt(225.0), abs=0)


def test_python_flatten_matches_cpp_flatten():
    world, lights, _ = rtw.scenes.simple(0x5EED0001)
    soa, _ = rtw.scenes.simple_soa(0x5EED0001)
    flat = rtw.flatten(world, lights)
    for f in ("spheres", "sphere_mat", "planes", "plane_mat", "mat_type", "mat_params", "lights"):
        np.testing.assert_array_equal(getattr(flat, f), getattr(soa, f), err_msg=f)


def test_encode_rgb8_matches_write_colour():
    """colour.rs:14-36: sqrt(sum/spp), clamp, (256 x) as u8 saturating, NaN -> 0;
    main.rs:97-104 writes the rows top (j = H-1) first."""
    sums = np.array([[[0.0, 1.0, 4.0], [np.nan, -1.0, 1e9]],
                     [[0.999 * 4, 0.25 * 4, np.inf]]] * 1, dtype=object)
    sums = np.array([[[0.0, 1.0, 4.0], [np.nan, -1.0, 1e9]],
                     [[3.996, 1.0, np.inf], [2.0, 0.04, 0.0]]], np.float64)
    out = rtw.encode_rgb8(sums, 4)

    def ref(x):
        v = np.sqrt(x / 4) if x >= 0 else np.nan
        if np.isnan(v):
            return 0
        return min(255, int(256 * min(max(v, 0.0), 1.0)))

    for r in range(2):
        j = 1 - r
        for i in range(2):
            assert list(out[r, i]) == [ref(x) for x in sums[j, i]]


def _write_colour(x, spp):
    """colour.rs:14-36 restated in Python floats (IEEE f64): scale =
    (spp as f64).recip(); (256 * sqrt(x * scale).clamp(0, 1)) as u8 (Rust's
    float -> u8 cast saturates, NaN -> 0)."""
    scale = 1.0 / float(spp)
    v = math.sqrt(x * scale) if x * scale >= 0 else math.nan
    if v != v:
        return 0
    t = 256.0 * min(max(v, 0.0), 1.0)
    return 255 if t >= 255 else int(t)


def _boundary_cases(spp, limit=40):
    """sums next to an encoder step k/256 where x * (1/spp) and x / spp round
    to different u8 -- they pin the reciprocal multiply of colour.rs:24."""
    out = []
    for k in range(1, 256):
        x0 = spp * (k / 256) ** 2
        for direction in (-np.inf, np.inf):
            x = x0
            for _ in range(limit):
                x = float(np.nextafter(x, direction))
                if _write_colour(x, spp) != min(255, int(256 * min(1.0, math.sqrt(x / spp)))):
                    out.append(x)
    return out


@pytest.mark.parametrize("spp", [3, 100, 500])
def test_encode_rgb8_values_pin_the_recip_multiply(spp):
    """Random sums and sums at the u8 step boundaries, at spp 3 / 100 / 500;
    at spp 3 and 500 there are sums where sum * (1/spp) and sum / spp encode
    differently, and the encoder must follow the reference's recip."""
    rng = np.random.default_rng(spp)
    vals = list(rng.uniform(0, 1.2 * spp, 3000)) + list(rng.uniform(0, 0.01 * spp, 3000))
    edge = _boundary_cases(spp)
    if spp in (3, 500):
        assert edge, "expected sums that tell x*(1/spp) from x/spp apart"
    vals = np.array((vals + edge + [0.0, -1.0, np.nan, np.inf, spp * 1.0])[: 3 * ((len(vals) + len(edge) + 5) // 3)])
    vals = np.concatenate([vals, np.zeros((-len(vals)) % 3)])
    sums = vals.reshape(1, -1, 3)
    out = rtw.encode_rgb8(sums, spp)
    want = np.array([_write_colour(x, spp) for x in vals], np.uint8).reshape(1, -1, 3)
    np.testing.assert_array_equal(out, want)


def test_encode_rgb8_f32_sums_widen_exactly():
    """A speed-mode (f32) framebuffer encodes as its exact f64 values would."""
    rng = np.random.default_rng(5)
    sums = rng.uniform(-1, 600, (7, 9, 3)).astype(np.float32)
    sums[0, 0] = [np.nan, np.inf, 0.0]
    np.testing.assert_array_equal(rtw.encode_rgb8(sums, 500), rtw.encode_rgb8(sums.astype(np.float64), 500))


def test_write_ppm_f32_matches_f64(tmp_path):
    sums = np.random.default_rng(6).uniform(0, 120, (5, 4, 3)).astype(np.float32)
    a, b = tmp_path / "a.ppm", tmp_path / "b.ppm"
    rtw.write_ppm(str(a), sums, 100)
    rtw.write_ppm(str(b), sums.astype(np.float64), 100)
    assert a.read_bytes() == b.read_bytes()


def test_write_ppm_layout(tmp_path):
    sums = np.zeros((2, 3, 3))
    sums[0, :, 0] = 4.0          # bottom row red
    p = tmp_path / "image.ppm"
    rtw.write_ppm(str(p), sums, 4)
    lines = p.read_text().splitlines()
    assert lines[:3] == ["P3", "3 2", "255"]
    assert lines[3:6] == ["0 0 0"] * 3 and lines[6:9] == ["255 0 0"] * 3


def test_renderer_without_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(rtw.RenderError):
        rtw.Renderer()


def test_kernel_isa_identity_covers_every_render_kernel_variant():
    """isa.py finds the gfx950 machine code of the launched variants by name
    (bench.py ties the committed PMC profiles to it): the headline f32 hit64
    kernel and the f64 parity kernel have distinct, stable hashes."""
    from ray_tracing_weekend_amd import isa
    h32 = isa.kernel_isa_sha(isa.render_kernel_symbol("f32", 5, 16))
    h64 = isa.kernel_isa_sha(isa.render_kernel_symbol("f64", 5, 0))
    assert h32 and h64 and h32 != h64 and len(h32) == 16
    assert isa.kernel_isa_sha(isa.render_kernel_symbol("f32", 5, 16)) == h32
    name = isa.render_kernel_name("f32", 5, 16)
    assert name == "void rtw::dev::render_kernel<float, 5, 16>(rtw::KParams<float>)"
    assert isa.demangled_to_symbol(name) == isa.render_kernel_symbol("f32", 5, 16)
    assert isa.kernel_isa_sha("_ZN3rtw3dev13no_such_kernelEv") is None


def test_device_list_arguments_refused_before_any_hip_call():
    """ABI 9: rtw_create_virtual / rtw_create_mask_ex / rtw_create_devices
    reject bad arguments with RTW_E_INVALID before touching HIP (no GPU
    here); rtw_visible_devices reports no device (or a HIP error) on this host."""
    lib = rtw._lib
    out = C.c_void_p()
    inv = _capi.RTW_E_INVALID
    assert lib.rtw_create_virtual(0, 0, _capi.RTW_F64, C.byref(out)) == inv          # no ranks
    assert lib.rtw_create_virtual(-1, 2, _capi.RTW_F64, C.byref(out)) == inv         # negative device
    assert lib.rtw_create_virtual(0, 2, 7, C.byref(out)) == inv                      # bad precision
    assert lib.rtw_create_virtual(0, 65, _capi.RTW_F64, C.byref(out)) == inv         # more ranks than the ABI allows
    assert lib.rtw_create_virtual(0, 2, _capi.RTW_F64, None) == inv
    assert lib.rtw_create_mask_ex(0, _capi.RTW_F64, C.byref(out)) == inv             # empty mask
    assert lib.rtw_create_mask_ex(1, 7, C.byref(out)) == inv
    devs = (C.c_int * 2)(0, 0)
    assert lib.rtw_create_devices(devs, 2, _capi.RTW_F64, C.byref(out)) == inv       # repeated device
    assert out.value is None
    assert lib.rtw_visible_devices() <= 0
    st = _capi.rtw_stats()
    assert lib.rtw_get_stats_rank(None, 0, C.byref(st)) == inv
