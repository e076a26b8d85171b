"""CPU check of the f32-vs-f64 statistics (tests/f32_stats.py) on synthetic
Monte-Carlo images: an unbiased renderer reads as noise, a 1 % image bias and
a regional bias are caught."""
import numpy as np

import f32_stats


def _renders(rng, truth, spp, bias=None):
    def one():
        # per-pixel mean of spp exponential samples around the truth
        return rng.gamma(spp, truth / spp)[..., None].repeat(3, -1)
    x = one()
    if bias is not None:
        x = x * bias[..., None]
    return x, one(), one()


def test_unbiased_reads_as_noise():
    rng = np.random.default_rng(1)
    truth = rng.uniform(0.1, 1.0, (160, 240))
    s = f32_stats.compare(*_renders(rng, truth, 64))
    assert abs(s["mean_bias_z"]) < 5 and abs(s["mean_rel_bias"]) < 2e-3
    assert 0.9 < s["msd_ratio"] < 1.1
    assert s["block_z_p99"] < 4.0 and 0.8 < s["block_z_rms"] < 1.2
    assert s["pixel_z_p99"] < 1.1 * s["pixel_z_p99_f64_seeds"]


def test_global_bias_is_caught():
    rng = np.random.default_rng(2)
    truth = rng.uniform(0.1, 1.0, (160, 240))
    s = f32_stats.compare(*_renders(rng, truth, 64, bias=np.full(truth.shape, 0.99)))
    assert abs(s["mean_rel_bias"] + 0.01) < 2e-3 and s["mean_bias_z"] < -10


def test_regional_bias_is_caught():
    rng = np.random.default_rng(3)
    truth = rng.uniform(0.1, 1.0, (160, 240))
    bias = np.ones(truth.shape)
    bias[32:64, 48:96] = 0.9
    s = f32_stats.compare(*_renders(rng, truth, 64, bias=bias))
    assert s["block_z_max"] > 6 and s["block_z_p99"] > 4


def test_nan_fractions():
    rng = np.random.default_rng(4)
    truth = rng.uniform(0.1, 1.0, (64, 64))
    a, b, c = _renders(rng, truth, 16)
    a[:2] = np.nan
    s = f32_stats.compare(a, b, c)
    assert abs(s["nan_frac_f32"] - 2 / 64) < 1e-12 and s["nan_frac_f64"] == 0.0
