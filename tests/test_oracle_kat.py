"""Known-answer tests that pin the CPU oracle (oracle/) to the reference's
formulas.  The reference's own tests hold no numeric fixtures
(integration-tests/src/lib.rs:7-112 only check "does not panic") and the Rust
reference cannot be built here, so the oracle is pinned by (a) hand-derived
values from the cited formulas, (b) independent pure-Python restatements of
the published algorithms it uses (xoshiro256++, splitmix64, rand 0.8.6's
float/int distributions), (c) Monte-Carlo identities of its samplers, and (d)
the committed golden renders (tests/golden/make_golden.py)."""
import json
import math
import os
import struct

import numpy as np
import pytest

from oracle import oracle as O

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
M64 = (1 << 64) - 1


def arr(*v):
    return (O.C.c_double * len(v))(*v)


# ---------------------------------------------------------------- RNG (pure Python restatements)
def mix64(z):
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def rotl(x, k):
    return ((x << k) | (x >> (64 - k))) & M64


class PyXoshiro:
    def __init__(self, s):
        self.s = list(s)

    def next(self):
        s = self.s
        result = (rotl((s[0] + s[3]) & M64, 23) + s[0]) & M64
        t = (s[1] << 17) & M64
        s[2] ^= s[0]
        s[3] ^= s[1]
        s[1] ^= s[2]
        s[0] ^= s[3]
        s[2] ^= t
        s[3] = rotl(s[3], 45)
        return result


def py_seed(seed, pix, samp):
    k = mix64((seed + 0x9E3779B97F4A7C15 * (pix + 1)) & M64)
    k = mix64(k ^ ((0xD1B54A32D192ED03 * (samp + 1)) & M64))
    st = []
    for _ in range(4):
        k = (k + 0x9E3779B97F4A7C15) & M64
        st.append(mix64(k))
    return st


def test_splitmix64_published_vector():
    # Vigna's splitmix64 with state 0: first output 0xE220A8397B1DCDAF
    assert mix64(0x9E3779B97F4A7C15) == 0xE220A8397B1DCDAF


def test_xoshiro256pp_first_output_by_hand():
    # state {1, 2, 3, 4}: result = rotl(1 + 4, 23) + 1 = 5 * 2^23 + 1
    assert PyXoshiro([1, 2, 3, 4]).next() == 41943041


@pytest.mark.parametrize("seed,pix,samp", [(0, 0, 0), (0x5EED0001, 12345, 7), (M64, 2**40, 499)])
def test_oracle_rng_matches_python_restatement(seed, pix, samp):
    r = O.Rng(seed, pix, samp)
    assert list(r.st) == py_seed(seed, pix, samp)
    py = PyXoshiro(py_seed(seed, pix, samp))
    for _ in range(64):
        assert r.next_u64() == py.next()


def test_rand_float_distributions_match_rand_0_8_6():
    r = O.Rng(9, 1, 2)
    py = PyXoshiro(py_seed(9, 1, 2))
    for _ in range(200):
        # Standard: (v >> 11) * 2^-53
        assert r.std() == (py.next() >> 11) * 2.0 ** -53
        # Open01: 52-bit fraction into [1, 2), minus (1 - EPSILON / 2)
        v = py.next()
        f = struct.unpack("<d", struct.pack("<Q", (v >> 12) | 0x3FF0000000000000))[0]
        x = r.open01()
        assert x == f - (1.0 - 2.0 ** -53) and 0.0 < x < 1.0
        # Uniform::new_inclusive(-0.5, 0.5): scale = 1 / (1 - 2^-52), value0_1 * scale + low
        v = py.next()
        f = struct.unpack("<d", struct.pack("<Q", (v >> 12) | 0x3FF0000000000000))[0] - 1.0
        scale = 1.0 / (1.0 - 2.0 ** -52)
        while scale * (1.0 - 2.0 ** -52) + -0.5 > 0.5:
            scale = np.nextafter(scale, 0.0)
        u = r.uniform_incl(-0.5, 0.5)
        assert u == f * scale + -0.5 and -0.5 <= u <= 0.5


@pytest.mark.parametrize("n", [1, 2, 3, 19, 25, 1000, 2**31 + 5])
def test_gen_index_widening_multiply(n):
    """gen_range(0..n) for u32: v = next_u64 >> 32; (hi, lo) = v * n; accept lo <= zone."""
    r = O.Rng(4, 4, 4)
    py = PyXoshiro(py_seed(4, 4, 4))
    zone = ((n << (32 - n.bit_length())) & 0xFFFFFFFF) - 1
    for _ in range(100):
        got = r.index(n)
        while True:
            v = py.next() >> 32
            m = v * n
            if (m & 0xFFFFFFFF) <= zone:
                assert got == m >> 32
                break


def test_sincos_2pi_accuracy_and_exact_quadrants():
    s, c = O.C.c_double(), O.C.c_double()
    for r, es, ec in [(0.0, 0.0, 1.0), (0.25, 1.0, 0.0), (0.5, 0.0, -1.0), (0.75, -1.0, 0.0)]:
        O.lib().rtwo_sincos_2pi(r, O.C.byref(s), O.C.byref(c))
        assert abs(s.value - es) < 1e-16 and abs(c.value - ec) < 1e-16
    rng = np.random.default_rng(0)
    worst = 0.0
    for r in rng.random(2000):
        O.lib().rtwo_sincos_2pi(float(r), O.C.byref(s), O.C.byref(c))
        worst = max(worst, abs(s.value - math.sin(2 * math.pi * r)), abs(c.value - math.cos(2 * math.pi * r)))
    assert worst < 1.5e-15   # the reference value carries the rounding of 2*pi*r itself


# ---------------------------------------------------------------- primitives
def sphere_hit(sph, o, d, tmin=2.220446049250313e-16, tmax=math.inf):
    t, n, f = O.C.c_double(), (O.C.c_double * 3)(), O.C.c_int()
    hit = O.lib().rtwo_sphere_hit(arr(*sph), arr(*o), arr(*d), tmin, tmax, O.C.byref(t), n, O.C.byref(f))
    return (t.value, list(n), f.value) if hit else None


def test_sphere_hit_near_root_and_front_face():
    # sphere.rs:61-99: |d| = 2 (directions are not normalised), near root t = 2
    t, n, front = sphere_hit((0, 0, -5, 1), (0, 0, 0), (0, 0, -2))
    assert t == 2.0 and n == [0, 0, 1] and front == 1


def test_sphere_hit_from_inside_takes_far_root_and_flips_normal():
    t, n, front = sphere_hit((0, 0, 0, 2), (0, 0, 0), (1, 0, 0))
    assert t == 2.0 and front == 0 and n == [-1, 0, 0]


def test_sphere_behind_tangent_and_range_inclusive():
    assert sphere_hit((0, 0, 5, 1), (0, 0, 0), (0, 0, -1)) is None          # behind
    assert sphere_hit((0, 1, -5, 1), (0, 0, 0), (0, 0, -1)) is None         # tangent: disc == 0
    t, _, _ = sphere_hit((0, 0, -5, 1), (0, 0, 0), (0, 0, -1), tmin=4.0)    # root == tmin: hit
    assert t == 4.0
    t, _, _ = sphere_hit((0, 0, -5, 1), (0, 0, 0), (0, 0, -1), tmin=4.5)    # near root excluded
    assert t == 6.0


def test_plane_is_one_sided():
    """plane.rs:61-76: hit only when the ray moves along +n (d.n > EPS)."""
    t, n, f = O.C.c_double(), (O.C.c_double * 3)(), O.C.c_int()
    pl = arr(0, 0, 0, 0, 1, 0)
    assert not O.lib().rtwo_plane_hit(pl, arr(0, 5, 0), arr(0, -1, 0), 1e-16, math.inf, O.C.byref(t), n, O.C.byref(f))
    assert O.lib().rtwo_plane_hit(pl, arr(0, -3, 0), arr(0, 2, 0), 1e-16, math.inf, O.C.byref(t), n, O.C.byref(f))
    assert t.value == 1.5 and f.value == 0 and list(n) == [0, -1, 0]


def test_aabb_slab():
    box = arr(-1, -1, -1, 1, 1, 1)
    lib = O.lib()
    assert lib.rtwo_aabb_hit(box, arr(0, 0, -5), arr(0, 0, 1), 0.0, math.inf)
    assert not lib.rtwo_aabb_hit(box, arr(0, 3, -5), arr(0, 0, 1), 0.0, math.inf)
    assert not lib.rtwo_aabb_hit(box, arr(0, 0, -5), arr(0, 0, 1), 0.0, 3.0)       # range ends first
    assert lib.rtwo_aabb_hit(box, arr(0, 0, 0), arr(0.3, -0.2, 1), 0.0, math.inf)  # origin inside
    # the plane's AABB pins y at 0 wherever the plane is (plane.rs:218-242)
    flat = arr(-math.inf, 0, -math.inf, math.inf, 0, math.inf)
    assert lib.rtwo_aabb_hit(flat, arr(0, 1, 0), arr(0, -1, 0), 1e-16, math.inf)
    assert not lib.rtwo_aabb_hit(flat, arr(0, -1, 0), arr(0, -1, 0), 1e-16, math.inf)


def test_onb_positive_x_normal_is_finite_and_orthonormal():
    """geometry/src/onb.rs:38-60."""
    u, v, w = (O.C.c_double * 3)(), (O.C.c_double * 3)(), (O.C.c_double * 3)()
    for nrm in [(1, 0, 0), (0, 0, 3), (-0.2, 5, 1)]:
        O.lib().rtwo_onb(arr(*nrm), u, v, w)
        m = np.array([list(u), list(v), list(w)])
        assert np.all(np.isfinite(m))
        np.testing.assert_allclose(m @ m.T, np.eye(3), atol=1e-15)
        np.testing.assert_allclose(m[2], np.array(nrm) / np.linalg.norm(nrm), atol=1e-15)


def test_schlick_reflectance():
    """material.rs:450-454, uses the ratio passed in (not the ior)."""
    lib = O.lib()
    assert abs(lib.rtwo_reflectance(1.0, 1.0 / 1.5) - 0.04) < 1e-15
    assert lib.rtwo_reflectance(0.0, 1.0 / 1.5) == 1.0
    x = 0.7
    r0 = ((1 - 1.5) / (1 + 1.5)) ** 2
    assert abs(lib.rtwo_reflectance(x, 1.5) - (r0 + (1 - r0) * (1 - x) ** 5)) < 1e-15


def test_reflect_refract_identities():
    out = (O.C.c_double * 3)()
    O.lib().rtwo_reflect(arr(1, -1, 0), arr(0, 1, 0), out)
    assert list(out) == [1, 1, 0]
    O.lib().rtwo_refract(arr(0, -1, 0), arr(0, 1, 0), 1 / 1.5, out)
    assert list(out) == [0, -1, 0]                                   # normal incidence
    s = math.sin(math.radians(30))
    v = (s, -math.cos(math.radians(30)), 0)
    O.lib().rtwo_refract(arr(*v), arr(0, 1, 0), 1 / 1.5, out)        # Snell: sin t = sin i / 1.5
    assert abs(out[0] - s / 1.5) < 1e-15 and abs(np.linalg.norm(list(out)) - 1) < 1e-15


def test_sphere_pdf_is_inverse_solid_angle_and_nan_inside():
    """sphere.rs:101-111: 1 / (2 pi (1 - sqrt(1 - r^2/d^2))); NaN from inside (sqrt of < 0)."""
    lib = O.lib()
    sph = arr(0, 0, -10, 2)
    v = lib.rtwo_sphere_pdf_value(sph, arr(0, 0, 0), arr(0, 0, -1))
    assert abs(v - 1 / (2 * math.pi * (1 - math.sqrt(1 - 4 / 100)))) < 1e-15
    assert lib.rtwo_sphere_pdf_value(sph, arr(0, 0, 0), arr(0, 1, 0)) == 0.0
    assert math.isnan(lib.rtwo_sphere_pdf_value(sph, arr(0, 0, -9.5), arr(1, 0, 0)))
    out = (O.C.c_double * 3)()
    r = O.Rng(1, 1, 1)
    lib.rtwo_sphere_random(sph, arr(0, 0, -10.5), r.st, out)
    assert all(math.isnan(x) for x in out)


def test_sphere_random_directions_hit_the_sphere():
    lib = O.lib()
    sph = arr(3, 1, -7, 1.5)
    out = (O.C.c_double * 3)()
    r = O.Rng(2, 3, 4)
    for _ in range(500):
        lib.rtwo_sphere_random(sph, arr(0, 0, 0), r.st, out)
        assert lib.rtwo_sphere_pdf_value(sph, arr(0, 0, 0), out) > 0


def test_samplers_moments():
    lib = O.lib()
    r = O.Rng(5, 6, 7)
    out = (O.C.c_double * 3)()
    cz, us = [], []
    for _ in range(20000):
        lib.rtwo_cosine_hemisphere(r.st, out)
        cz.append(out[2])
        lib.rtwo_unit_sphere(r.st, out)
        us.append(list(out))
    cz, us = np.array(cz), np.array(us)
    # cosine-weighted hemisphere: z = cos(theta) >= 0, E[z] = 2/3, |v| = 1
    assert cz.min() >= 0 and abs(cz.mean() - 2 / 3) < 0.01
    # uniform ball: |x| < 1, E[|x|^2] = 3/5, E[x] = 0
    n2 = (us ** 2).sum(1)
    assert n2.max() < 1 and abs(n2.mean() - 0.6) < 0.01 and np.all(np.abs(us.mean(0)) < 0.02)


# ---------------------------------------------------------------- whole-path checks
def test_empty_world_returns_background_sums():
    sc = O.Scene(np.zeros((0, 4)), np.zeros(0, np.uint32), np.zeros((0, 6)), np.zeros(0, np.uint32),
                 np.zeros(0, np.uint32), np.zeros((0, 5)), np.zeros((0, 4)))
    cam = O.camera_build(image_width=5, image_height=4, samples_per_pixel=7, background=(0.5, 0.25, 1.0))
    img, st = O.render(cam, sc, 1)
    np.testing.assert_array_equal(img, np.broadcast_to([3.5, 1.75, 7.0], img.shape))
    assert st.segments == 5 * 4 * 7


def test_lambertian_without_lights_panics_when_the_light_branch_is_drawn():
    """HittableList::random on an empty list panics (hittable_list.rs:414-419)
    -- only when MixturePdf::generate picks the light half (pdf.rs:94-100);
    a scene whose Lambertian surfaces are never hit renders fine (the
    reference's `plane` scene)."""
    sc = O.Scene(np.array([[0, 0, -1, 0.5]]), np.array([0], np.uint32), np.zeros((0, 6)),
                 np.zeros(0, np.uint32), np.array([0], np.uint32), np.array([[0.5, 0.5, 0.5, 0, 0]]),
                 np.zeros((0, 4)))
    with pytest.raises(O.ReferencePanic) as e:
        O.render(O.camera_build(image_width=4, image_height=4, samples_per_pixel=8), sc, 1)
    st = e.value.stats
    assert 0 < st.panic_no_lights < st.lambertian and st.panic_plane_uv == 0
    # the cosine half divides by the empty list's 0 / 0 pdf: NaN samples
    img, st = O.render(O.camera_build(image_width=4, image_height=4, samples_per_pixel=8), sc, 1,
                       allow_panic=True)
    assert st.nan_samples >= st.panic_no_lights
    # never hit: no panic, background only
    cam = O.camera_build(image_width=3, image_height=2, samples_per_pixel=4, lookat=(0, 0, 1),
                         background=(0.5, 0.25, 1.0))
    img, st = O.render(cam, sc, 1)
    assert st.lambertian == 0 and np.all(img == np.array([2.0, 1.0, 4.0]))


def test_bvh_variants_equal_brute_force():
    """bvh.rs:164-188 keeps 'closest hit over every primitive': the restated
    reference BVH (with and without its per-visit node-AABB recomputation)
    must give the brute-force image bit for bit."""
    sc = O.scene_simple(0x5EED0001)
    cam = O.camera_build(**dict(O.simple_camera_kw(), image_width=24, image_height=16,
                                samples_per_pixel=3, max_depth=50))
    imgs = [O.render(cam, sc, 77, accel=a)[0] for a in (O.ACCEL_BRUTE, O.ACCEL_BVH_REF, O.ACCEL_BVH_CACHED)]
    for im in imgs[1:]:
        assert np.array_equal(np.nan_to_num(imgs[0], nan=-7), np.nan_to_num(im, nan=-7))


def test_reference_bvh_shape():
    sc = O.scene_simple(0x5EED0001)
    nodes, leaves, depth = O.bvh_stats(sc)
    assert nodes == 2 * leaves - 1 and leaves >= (len(sc.sphere_mat) + 1) / 5 and depth < 20


def test_two_seeds_converge_to_the_same_image():
    """Statistical convergence: per-pixel means of two independent seeds agree
    (NaN-free pixels), i.e. the estimator has no seed-dependent bias."""
    sc = O.scene_simple(0x5EED0001)
    spp = 64
    cam = O.camera_build(**dict(O.simple_camera_kw(), image_width=32, image_height=18,
                                samples_per_pixel=spp, max_depth=50))
    a, _ = O.render(cam, sc, 1, accel=O.ACCEL_BVH_CACHED)
    b, _ = O.render(cam, sc, 2, accel=O.ACCEL_BVH_CACHED)
    ok = ~(np.isnan(a).any(-1) | np.isnan(b).any(-1))
    ma, mb = a[ok].mean() / spp, b[ok].mean() / spp
    assert abs(ma - mb) < 0.01 * ma


def test_golden_scene_fixture():
    g = json.load(open(os.path.join(GOLDEN, "simple_scene_5EED0001.json")))
    sc = O.scene_simple(g["seed"])
    for k in ("spheres", "sphere_mat", "planes", "plane_mat", "mat_type", "mat_params", "lights"):
        np.testing.assert_array_equal(np.asarray(getattr(sc, k)), np.asarray(g[k]), err_msg=k)


def test_golden_renders_reproduce():
    import importlib.util
    spec = importlib.util.spec_from_file_location("mg", os.path.join(GOLDEN, "make_golden.py"))
    mg = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mg)
    data = np.load(os.path.join(GOLDEN, "golden_renders.npz"))
    sc = O.scene_simple(mg.SCENE_SEED)
    for name, over, chunk, rows, cols in mg.CASES:
        kw = dict(O.simple_camera_kw())
        kw.update(over)
        img, _ = O.render(O.camera_build(**kw), sc, mg.RENDER_SEED, chunk=chunk,
                          accel=O.ACCEL_BRUTE, rows=rows, cols=cols)
        if rows is not None:
            img = img[rows[0]:rows[1], cols[0]:cols[1]]
        assert np.array_equal(np.nan_to_num(img, nan=-7), np.nan_to_num(data[name], nan=-7)), name


# ---- Quad + DiffuseLight (quadrilateral.rs, material.rs:490-514)

QUAD = (0.0, 0.0, 0.0, 2.0, 0.0, 0.0, 0.0, 0.0, 3.0)      # Q, u, v: the y = 0 plane, 2 x 3


def test_quad_new_aabb_pads_the_flat_axis():
    """Quad::new: AABBox::from_points([q + (u+v)/2, q, q+v, q+u, q+u+v]), each
    enclose padding axes thinner than 1e-4 by 1e-4 (aabox.rs:129-149)."""
    lo, hi = O.quad_aabb(QUAD)
    assert lo == (0.0, -1e-4, 0.0) and hi == (2.0, 1e-4, 3.0)


def test_quad_hit_is_two_sided_with_uv_and_front_face():
    # normal = u x v / |u x v| = (0, -1, 0); from above the ray is a back hit
    t, a, b, n = O.quad_hit(QUAD, (1.0, 1.0, 1.0), (0.0, -1.0, 0.0))
    assert (t, a, b) == (1.0, 0.5, 1.0 / 3.0) and n == (-0.0, 1.0, -0.0)
    t, a, b, n = O.quad_hit(QUAD, (1.0, -2.0, 1.5), (0.0, 1.0, 0.0))
    assert (t, a, b) == (2.0, 0.5, 0.5) and n == (0.0, -1.0, 0.0)


def test_quad_hit_uv_range_inclusive_and_parallel_miss():
    assert O.quad_hit(QUAD, (2.0, 1.0, 3.0), (0.0, -1.0, 0.0))[1:3] == (1.0, 1.0)   # corner
    assert O.quad_hit(QUAD, (0.0, 1.0, 0.0), (0.0, -1.0, 0.0))[1:3] == (0.0, 0.0)
    assert O.quad_hit(QUAD, (2.5, 1.0, 1.0), (0.0, -1.0, 0.0)) is None            # alpha > 1
    assert O.quad_hit(QUAD, (1.0, 1.0, 1.0), (1.0, 0.0, 0.0)) is None             # |d.n| <= EPS
    assert O.quad_hit(QUAD, (1.0, 1.0, 1.0), (0.0, -1.0, 0.0), tmax=0.5) is None  # t outside range


def test_quad_pdf_is_distance_squared_over_cosine_area():
    o, d = (0.0, 4.0, 0.0), (1.0, -2.0, 1.5)            # hits (2, 0, 3)... at t = 2 -> (2, 0, 3)
    t, _, _, _ = O.quad_hit(QUAD, o, d, 0.0)
    assert t == 2.0
    d2 = t * t * (1 + 4 + 2.25)
    cosine = abs(-2.0) / math.sqrt(1 + 4 + 2.25)
    assert O.quad_pdf_value(QUAD, o, d) == pytest.approx(d2 / (cosine * 6.0), rel=1e-15)
    assert O.quad_pdf_value(QUAD, o, (0.0, 1.0, 0.0)) == 0.0


def test_quad_random_is_q_plus_open01_u_and_v():
    r1, r2 = O.Rng(5, 6, 7), O.Rng(5, 6, 7)
    o = (0.5, 1.0, -2.0)
    x = O.quad_random(QUAD, o, r1)
    a, b = r2.open01(), r2.open01()                      # u's draw first (quadrilateral.rs:115-116)
    assert x == (2.0 * a - 0.5, -1.0, 3.0 * b + 2.0)


def _quad_scene(light_rgb=(4.0, 2.0, 1.0)):
    """A DiffuseLight quad facing a camera, nothing else."""
    return O.Scene(np.zeros((0, 4)), np.zeros(0, np.uint32), np.zeros((0, 6)), np.zeros(0, np.uint32),
                   np.array([4], np.uint32), np.array([[*light_rgb, 0.0, 0.0]]), np.zeros((0, 4)),
                   quads=np.array([[-5.0, -5.0, -3.0, 10.0, 0.0, 0.0, 0.0, 10.0, 0.0]]),
                   quad_mat=np.array([0], np.uint32))


def test_diffuse_light_emits_its_colour_and_stops():
    """scatter() is None for DiffuseLight: the sample is mult * emitted + res
    with mult = 1 (camera.rs:484-486) -- exactly the light's colour."""
    cam = O.camera_build(image_width=4, image_height=3, samples_per_pixel=5, max_depth=10,
                         background=(0.0, 0.0, 0.0))
    img, st = O.render(cam, _quad_scene(), 3)
    np.testing.assert_array_equal(img, np.broadcast_to([20.0, 10.0, 5.0], img.shape))
    assert st.segments == 4 * 3 * 5 and st.lambertian == 0


def test_quad_world_bvh_variants_equal_brute_force():
    """Quads join the BVH as a third type group; closest hit must not change."""
    rng = np.random.default_rng(2)
    quads = np.concatenate([rng.uniform(-3, 3, (20, 3)), rng.uniform(-1, 1, (20, 6))], axis=1)
    sph = np.concatenate([rng.uniform(-3, 3, (30, 3)), rng.uniform(0.1, 0.5, (30, 1))], axis=1)
    mats = np.array([0, 1, 2, 4], np.uint32)
    mp = np.array([[0.6, 0.5, 0.4, 0, 0], [0.8, 0.8, 0.8, 0.2, 0], [1, 1, 1, 0, 1.5], [3, 3, 3, 0, 0]])
    sc = O.Scene(sph, rng.integers(0, 4, 30).astype(np.uint32), np.zeros((0, 6)), np.zeros(0, np.uint32),
                 mats, mp, np.array([[0.0, 4.0, 0.0, 1.0]]), quads=quads,
                 quad_mat=rng.integers(0, 4, 20).astype(np.uint32),
                 light_quads=quads[:2], light_kinds=np.array([1, 0, 1], np.uint32))
    cam = O.camera_build(image_width=16, image_height=12, samples_per_pixel=3, max_depth=20,
                         lookfrom=(0.0, 2.0, 9.0), lookat=(0.0, 0.0, 0.0), background=(0.5, 0.6, 0.7))
    imgs = [O.render(cam, sc, 9, accel=a)[0] for a in (O.ACCEL_BRUTE, O.ACCEL_BVH_REF, O.ACCEL_BVH_CACHED)]
    for im in imgs[1:]:
        np.testing.assert_array_equal(np.nan_to_num(im, nan=-7), np.nan_to_num(imgs[0], nan=-7))


# ---- Transformed<Cuboid> (cuboid.rs, entities/transformations.rs, geometry transformations.rs)

def _box(p, q, R=((1, 0, 0), (0, 1, 0), (0, 0, 1)), T=(0, 0, 0)):
    return list(p) + list(q) + [float(v) for row in R for v in row] + list(map(float, T))


def test_identity_box_is_the_cuboid_six_quads():
    b = _box((0, 0, 0), (2, 3, 4))
    t, p, n, front = O.box_hit(b, (1.0, 1.0, -5.0), (0.0, 0.0, 1.0))
    # the min-z face is Quad(min_p, dx, dy): its normal dx x dy points +z, i.e.
    # INTO the cuboid, so this outside hit is a back face (cuboid.rs:38-45)
    assert t == 5.0 and p == (1.0, 1.0, 0.0) and not front and n == (0.0, 0.0, -1.0)
    # the quads' t from Quad::hit directly: the nearer face wins
    q0 = O.quad_hit((0, 0, 0, 2, 0, 0, 0, 3, 0), (1.0, 1.0, -5.0), (0.0, 0.0, 1.0))
    assert q0[0] == t


def test_translated_box_aabb_and_the_direction_translation():
    """Transformation::transform_vector3d ADDS the translation
    (geometry/src/transformations.rs:112-114): the inverse maps a direction d
    to R^-1 d - R^-1 T.  With a pure translation T the object-space ray is
    (o - T, d - T); its hit point goes back by + T."""
    T = (10.0, 0.0, 0.0)
    b = _box((0, 0, 0), (2, 2, 2), T=T)
    lo, hi = O.box_aabb(b)
    # AABBox::from_points pads after EVERY enclose: the first two corners
    # differ only in y, so x and z get 1e-4 twice at the low end
    assert all(a < b for a, b in zip(lo, (10.0, 0.0, 0.0))) and all(a > b for a, b in zip(hi, (12.0, 2.0, 2.0)))
    assert all(b - a < 5e-4 for a, b in zip(lo, (10.0, 0.0, 0.0)))
    o, d = (11.0, 1.0, -5.0), (10.0, 0.0, 1.0)          # object space: o' = (1, 1, -5), d' = (0, 0, 1)
    t, p, n, front = O.box_hit(b, o, d)
    assert t == 5.0 and p == (11.0, 1.0, 0.0) and n == (0.0, 0.0, -1.0) and not front


def test_singular_transformation_is_never_hit():
    b = _box((0, 0, 0), (1, 1, 1), R=((1, 0, 0), (0, 0, 0), (0, 0, 1)))   # det 0: inverse() is None
    assert O.box_hit(b, (0.5, 0.5, -3.0), (0.0, 0.0, 1.0)) is None


def test_transform_composition_matches_the_reference_order():
    """translate then rotate(15 deg, Y) = {R, R T} (apply: b.R * a.R, b.T + b.R * a.T)."""
    R, T = O.transform_compose(("translate", (265, 0, 295)), ("rotate", 15, 1))
    c, s = math.cos(15 * (math.pi / 180)), math.sin(15 * (math.pi / 180))
    assert R == [[c, 0.0, s], [0.0, 1.0, 0.0], [-s, 0.0, c]]
    assert T == [c * 265 + 0.0 * 0 + s * 295 + 0.0, 0.0, (-s * 265 + 0.0 * 0) + c * 295 + 0.0]


def test_cornell_coplanar_tie_goes_to_the_first_type_group():
    """The cuboid's bottom face lies in the floor's plane (y = 0): a ray
    reaching the floor under the box gets the same t from both.  The reference
    world is a flat HittableList whose hit is min_by over type groups in
    first-insertion order, Quad before Transformed<Cuboid>
    (hittable_list.rs:395-406; lib.rs:306-343), and min_by keeps the first
    minimum: the floor quad (object 2) wins."""
    import ray_tracing_weekend_amd as rtw
    soa, _ = rtw.scenes.cornell_box_soa()
    sc = O.Scene(**soa.__dict__)
    o = (404.1316009481821, 0.010599100747201926, 367.9403068786761)
    d = (-0.6518441571396578, -0.41416419117277475, 0.6352694054911589)
    k, t, p, n, front = O.world_hit(sc, o, d)
    assert k == 2 and p[1] == 0.0 and n == (-0.0, 1.0, -0.0) and not front
    # the box reports the same t for its own bottom face
    box = soa.boxes[0].tolist()
    assert O.box_hit(box, o, d)[0] == t
