"""Statistics of the f32 speed mode against the f64 parity mode (test
infrastructure: tests/test_gpu_f32_tolerance.py, tools/f32_tolerance.py).

The f32 mode draws the same RNG words as f64 but rounding separates the
paths (the reference's t_min = f64::EPSILON makes self-intersection chaotic,
camera.rs:473), so a per-pixel comparison at a FIXED seed measures Monte-Carlo
noise, not error.  The comparison here is two-sample: with three renders of
the same image -- f32 at seed X, f64 at seed Y (the reference: bit-identical to
the oracle, tested elsewhere) and f64 at seed Z -- the per-pixel differences
D32 = f32(X) - f64(Y) and D64 = f64(Z) - f64(Y) have the same distribution if
f32 is an unbiased, equally noisy renderer of the reference's image.  D64
therefore calibrates every statistic:

  mean_rel_bias   (mean f32 - mean f64) / mean f64 over the image, with its
                  z-score against the noise of a two-seed mean difference
  msd_ratio       mean D32^2 / mean D64^2 (extra variance or local bias > 1)
  block_z         16x16-pixel block means of D32 in units of their noise
                  (block std of D64 / 16, with an f32 rounding floor of
                  floor_rel x the block's value): a regional bias shows as |z| >> 1
  pixel_z_p99     99th percentile of |D32| / sigma_block, beside the same for D64
  nan fractions   of pixels whose sum is NaN (NaN samples are not scrubbed)

All images are per-pixel means (sum / spp), shape [H, W, 3].
"""
from __future__ import annotations

import numpy as np


def _blocks(a, b=16):
    h, w = a.shape[:2]
    h2, w2 = h - h % b, w - w % b
    return a[:h2, :w2].reshape(h2 // b, b, w2 // b, b, *a.shape[2:])


def compare(f32, f64_ref, f64_other, block=16, floor_rel=4e-6):
    nan32 = np.isnan(f32).any(-1)
    nan64 = np.isnan(f64_ref).any(-1)
    nan64o = np.isnan(f64_other).any(-1)
    ok = ~(nan32 | nan64 | nan64o)
    d32 = np.where(ok[..., None], f32 - f64_ref, 0.0)
    d64 = np.where(ok[..., None], f64_other - f64_ref, 0.0)
    n = int(ok.sum())
    out = {"pixels": int(ok.size), "pixels_compared": n,
           "nan_frac_f32": float(nan32.mean()), "nan_frac_f64": float(nan64.mean()),
           "nan_frac_f64_other": float(nan64o.mean())}
    m_ref = float(f64_ref[ok].mean())
    out["mean_f64"] = m_ref
    out["mean_f32"] = float(f32[ok].mean())
    out["mean_f64_other"] = float(f64_other[ok].mean())
    out["mean_rel_bias"] = float((f32[ok].mean() - m_ref) / m_ref)
    out["mean_rel_diff_f64_seeds"] = float((f64_other[ok].mean() - m_ref) / m_ref)
    # standard error of an image-mean difference of two independent renders:
    # the pixel-level spread of D64 (pixels are independent)
    se = float(d64[ok].mean(-1).std() / np.sqrt(max(n, 1)))
    out["mean_bias_z"] = float(d32[ok].mean() / se) if se > 0 else 0.0
    out["mean_diff_z_f64_seeds"] = float(d64[ok].mean() / se) if se > 0 else 0.0
    msd64 = float((d64[ok] ** 2).mean())
    out["msd_ratio"] = float((d32[ok] ** 2).mean() / msd64) if msd64 > 0 else 1.0
    # regional bias: block means of the (luminance-averaged) differences
    okb = _blocks(ok, block).astype(np.float64)
    cnt = okb.sum(axis=(1, 3))
    dd32 = _blocks(d32.mean(-1), block).sum(axis=(1, 3))
    dd64 = _blocks(d64.mean(-1), block)
    s64 = _blocks(d64.mean(-1) ** 2, block).sum(axis=(1, 3))
    good = cnt >= block * block // 2
    var64 = s64[good] / cnt[good]                     # E[D^2] per block (mean of D64 ~ 0)
    # + an f32 rounding floor: a block whose f64 pixels are (nearly) noise-free
    # -- the sky, where every sample is the background -- still differs by the
    # f32 rounding of the path products (floor_rel of the block's value)
    mref = _blocks(np.where(ok, f64_ref.mean(-1), 0.0), block).sum(axis=(1, 3))[good] / cnt[good]
    noise = np.sqrt(np.maximum(var64, 1e-300) / cnt[good] + (floor_rel * np.abs(mref)) ** 2)
    live = var64 > 0
    zb = dd32[good][live] / cnt[good][live] / noise[live]
    zb64 = dd64.sum(axis=(1, 3))[good][live] / cnt[good][live] / noise[live]
    out["blocks"] = int(live.sum())
    out["block_z_p99"] = float(np.percentile(np.abs(zb), 99)) if zb.size else 0.0
    out["block_z_max"] = float(np.abs(zb).max()) if zb.size else 0.0
    out["block_z_rms"] = float(np.sqrt((zb ** 2).mean())) if zb.size else 0.0
    out["block_z_p99_f64_seeds"] = float(np.percentile(np.abs(zb64), 99)) if zb64.size else 0.0
    out["block_z_rms_f64_seeds"] = float(np.sqrt((zb64 ** 2).mean())) if zb64.size else 0.0
    # per pixel, in units of the block's noise level
    sig = np.sqrt(np.maximum(s64 / np.maximum(cnt, 1), 1e-300))
    sig_px = np.repeat(np.repeat(sig, block, 0), block, 1)
    hh, ww = sig_px.shape
    okp = ok[:hh, :ww] & (np.repeat(np.repeat(good, block, 0), block, 1)) & (sig_px > 1e-150)
    z32 = np.abs(d32[:hh, :ww].mean(-1))[okp] / sig_px[okp]
    z64 = np.abs(d64[:hh, :ww].mean(-1))[okp] / sig_px[okp]
    out["pixel_z_p99"] = float(np.percentile(z32, 99)) if z32.size else 0.0
    out["pixel_z_p99_f64_seeds"] = float(np.percentile(z64, 99)) if z64.size else 0.0
    return out
