"""SURVEY.md §8(f) rank 1, end to end: a GPU render written by the product's
PPM writer (rtw_write_ppm, colour.rs:14-36 + bin/src/main.rs:89-104) is
byte-identical to the image.ppm that the oracle's sums give through an
independent Python restatement of the reference's writer.  f64 (the parity
mode: GPU sums == oracle sums bit for bit), spp 100 and 500."""
import math

import numpy as np
import pytest

import ray_tracing_weekend_amd as rtw
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _reference_ppm(sums, spp):
    """main.rs:89-104: "P3\\n{W} {H}\\n255\\n", then the rows from j = H-1 down
    to 0, each pixel "{r} {g} {b}\\n" via SampledColour's Display
    (colour.rs:14-36): scale = (spp as f64).recip(); (256 * sqrt(c * scale)
    .clamp(0, 1)) as u8 -- Rust's float -> int cast saturates, NaN -> 0."""
    H, W = sums.shape[:2]
    scale = 1.0 / float(spp)

    def u8(c):
        v = math.sqrt(c * scale) if c * scale >= 0 else math.nan
        if v != v:
            return 0
        t = 256.0 * min(max(v, 0.0), 1.0)
        return 255 if t >= 255 else int(t)

    out = [f"P3\n{W} {H}\n255\n"]
    for j in range(H - 1, -1, -1):
        for i in range(W):
            r, g, b = (u8(float(x)) for x in sums[j, i])
            out.append(f"{r} {g} {b}\n")
    return "".join(out).encode()


@pytest.mark.parametrize("spp", [100, 500])
def test_gpu_image_ppm_is_byte_identical(tmp_path, spp):
    soa, b = rtw.scenes.simple_soa(0x5EED0001)
    cam = b.with_image_width(64).with_image_height(36).with_samples_per_pixel(spp).with_max_depth(50).build()
    with rtw.Renderer(precision=rtw.RTW_F64) as r:
        r.set_tuning("partial_max", 1 << 30)
        r.set_scene(soa)
        gpu = r.render(cam, 77)
        chunk = int(r.stats.chunk)
    ocam = O.Camera()
    for name, _ in O.Camera._fields_:
        setattr(ocam, name, getattr(cam.raw, name))
    ref, _ = O.render(ocam, O.Scene(**soa.__dict__), 77, chunk=chunk, accel=O.ACCEL_BVH_CACHED)
    p = tmp_path / "image.ppm"
    n = rtw.write_ppm(str(p), gpu, spp)
    data = p.read_bytes()
    assert n == len(data)
    assert data == _reference_ppm(ref, spp)
