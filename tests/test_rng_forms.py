"""Bit identities the device RNG helpers rely on (CPU, numpy restatement of
the bit construction in csrc/rtw_device.hpp).

P<double>::u_pm1(v) replaces UnitSphere's coordinate 2 * u_std(v) - 1 (rand
0.8.6 Standard for f64 = (v >> 11) * 2^-53, utils.rs:99-122 as the oracle's
unit_sphere draws it) by D - (2 - b): D = the double with exponent 0 and the
52 mantissa bits 11..62 of v, b = bit 63.  Both forms must agree bit for bit,
signed zero included.  Rng::next's 64-bit rotations are built from two
32-bit funnel shifts (rotl<k>); checked against the plain shift form."""
import numpy as np


def _reference_form(v):
    u = (v >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)
    return 2.0 * u - 1.0


def _device_form(v):
    hi = (v >> np.uint64(32)).astype(np.uint32)
    lo = (v & np.uint64(0xFFFFFFFF)).astype(np.uint32)
    # v_alignbit(hi, lo, 11): bits 11..42 of v
    dlo = ((hi.astype(np.uint64) << np.uint64(21)) | (lo.astype(np.uint64) >> np.uint64(11))) & np.uint64(0xFFFFFFFF)
    dhi = np.uint32(0x3FF00000) | ((hi >> np.uint32(11)) & np.uint32(0xFFFFF))
    chi = np.uint32(0x40000000) - ((hi >> np.uint32(31)) << np.uint32(20))
    d = ((dhi.astype(np.uint64) << np.uint64(32)) | dlo).view(np.float64)
    c = (chi.astype(np.uint64) << np.uint64(32)).view(np.float64)
    return d - c


def test_u_pm1_matches_two_u_minus_one():
    rng = np.random.default_rng(7)
    v = rng.integers(0, 2**64 - 1, size=1 << 20, dtype=np.uint64, endpoint=True)
    edges = np.array([0, 1, 2**11 - 1, 2**11, 2**63 - 1, 2**63, 2**63 + 2**11, 2**64 - 1,
                      0x7FFFFFFFFFFFF800, 0x8000000000000000, 0xFFFFFFFFFFFFF800], dtype=np.uint64)
    v = np.concatenate([v, edges])
    a, b = _reference_form(v), _device_form(v)
    assert np.array_equal(a.view(np.uint64), b.view(np.uint64))
    assert a.min() == -1.0 and a.max() < 1.0
    # v = 2^63 gives +0 in both forms (not -0)
    z = _device_form(np.array([2**63], dtype=np.uint64))
    assert z[0] == 0.0 and not np.signbit(z[0])


def _alignbit(a, b, s):
    return np.uint32(((int(a) << 32 | int(b)) >> s) & 0xFFFFFFFF)


def _rotl_device(x, k):
    lo, hi = x & 0xFFFFFFFF, x >> 32
    if k < 32:
        return int(_alignbit(hi, lo, 32 - k)) << 32 | int(_alignbit(lo, hi, 32 - k))
    return int(_alignbit(lo, hi, 64 - k)) << 32 | int(_alignbit(hi, lo, 64 - k))


def test_rotl_as_two_alignbits():
    """Rng::next's rotations (xoshiro256++: 23 and 45) as rtw_device.hpp
    rotl<k> builds them from two 32-bit funnel shifts."""
    rng = np.random.default_rng(3)
    xs = [int(v) for v in rng.integers(0, 2**64 - 1, size=4000, dtype=np.uint64, endpoint=True)]
    xs += [0, 1, 2**63, 2**64 - 1, 0xFFFFFFFF, 0xFFFFFFFF00000000]
    m = (1 << 64) - 1
    for k in (1, 9, 23, 31, 33, 45, 63):
        for x in xs:
            assert _rotl_device(x, k) == ((x << k) | (x >> (64 - k))) & m, (x, k)
