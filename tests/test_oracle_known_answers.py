"""Pin the oracle (oracle/tray_oracle.c) against the reference's own known-answer
tests (fortio/tray ray/*_test.go) and the published Philox KAT vectors.
CPU only; no GPU, no product code."""
import math
import os

import numpy as np
import pytest

from conftest import DEFAULT_BG


def sphere(center, radius, material=1, albedo=(1, 0, 0), param=0.0):
    from oracle.oracle import SPHERE_DTYPE

    s = np.zeros(1, dtype=SPHERE_DTYPE)
    s["center"], s["radius"], s["albedo"], s["param"], s["material"] = center, radius, albedo, param, material
    return s


# ------------------------------------------------------------------ RNG -----
@pytest.mark.parametrize(
    "ctr,key,expected",
    [  # Random123 kat_vectors, philox4x32 R=10
        ((0, 0, 0, 0), (0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
        ((0xFFFFFFFF,) * 4, (0xFFFFFFFF,) * 2, (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
        ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
         (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1)),
    ],
)
def test_philox_kat(O, ctr, key, expected):
    assert O.philox4x32_10(ctr, key) == expected


def test_uniforms_range_and_resolution(O):
    us = np.array([O.uniforms(7, i, 0, 0, 3 << 24) for i in range(2000)]).ravel()
    assert us.min() >= 0.0 and us.max() < 1.0
    assert np.all(us * 2.0**53 == np.floor(us * 2.0**53))  # 53-bit grid


# ---------------------------------------------------------- vec3_test.go ----
@pytest.mark.parametrize(  # ray/vec3_test.go:764-787
    "v,expected",
    [((0, 0, 0), True), ((1e-9, 1e-10, 1e-11), True), ((1e-7, 0, 0), False), ((1, 2, 3), False),
     ((1e-9, 1e-9, 1e-6), False), ((-1e-10, -1e-11, -1e-12), True), ((1e-10, -1e-11, 1e-12), True)],
)
def test_near_zero(O, v, expected):
    assert O.near_zero(v) == expected


def test_reflect(O):  # ray/vec3_test.go:789-835 (1e-9)
    cases = [((1, -1, 0), (0, 1, 0), (1, 1, 0)), ((1, 1, 0), (1, 0, 0), (-1, 1, 0)),
             ((0, -1, 0), (0, 1, 0), (0, 1, 0)), (O.unit((1, -1, 0)), (0, 1, 0), O.unit((1, 1, 0)))]
    for v, n, e in cases:
        assert np.max(np.abs(O.reflect(v, n) - np.asarray(e))) <= 1e-9


def test_refract_bending(O):  # ray/vec3_test.go:837-904
    n = np.array([0.0, 1.0, 0.0])
    assert not O.near_zero(O.refract((0, -1, 0), n, 1.5))
    uv = O.unit((1, -1, 0))
    inc = math.acos(abs(np.dot(uv, n)))
    into = O.unit(O.refract(uv, n, 1.0 / 1.5))
    out = O.unit(O.refract(uv, n, 1.5))
    assert math.acos(abs(np.dot(into, n))) < inc  # entering glass bends toward the normal
    assert math.acos(abs(np.dot(out, n))) > inc   # exiting bends away


@pytest.mark.parametrize(  # ray/vec3_test.go:264-289 (ToSRGBA)
    "c,expected",
    [((0, 0, 0), (0, 0, 0)), ((1, 1, 1), (255, 255, 255)), ((1, 0, 0), (255, 0, 0)), ((0, 1, 0), (0, 255, 0)),
     ((0, 0, 1), (0, 0, 255)), ((0.5, 0.5, 0.5), (188, 188, 188)), ((1.5, 2.0, 3.0), (255, 255, 255)),
     ((-1.0, -0.5, -2.0), (0, 0, 0))],
)
def test_to_srgba(O, c, expected):
    assert tuple(O.to_srgba(np.array(c, dtype=float))[:3]) == expected
    assert O.to_srgba(np.array(c, dtype=float))[3] == 255


def test_random_unit_vector_length(O):  # ray/vec3_test.go:505-537 (1e-9)
    for i in range(200):
        assert abs(np.linalg.norm(O.unit_vector(42, i, 0, 0)) - 1.0) <= 1e-9


# ------------------------------------------------------- materials_test.go ---
@pytest.mark.parametrize("cosine,ref_idx", [(0.5, 1.5), (0.0, 1.5), (1.0, 1.5), (0.7, 1.33), (0.9, 2.0)])
def test_reflectance_schlick(O, cosine, ref_idx):  # ray/materials_test.go:205-231 (1e-10)
    r = O.reflectance(cosine, ref_idx)
    r0 = ((1 - ref_idx) / (1 + ref_idx)) ** 2
    assert 0 <= r <= 1
    assert abs(r - (r0 + (1 - r0) * (1 - cosine) ** 5)) <= 1e-10


def test_lambertian_scatter(O):  # ray/materials_test.go:8-31
    s = sphere((0, 0, 0), 1, 1, (0.5, 0.5, 0.5))
    ok, att, org, d = O.scatter(s, (0, 0, 0), (0, 0, -1), (0, 0, -1), (0, 0, 1), True)
    assert ok and tuple(att) == (0.5, 0.5, 0.5) and tuple(org) == (0, 0, -1)


def test_metal_scatter(O):  # ray/materials_test.go:33-82
    rd = O.unit((1, -1, 0))
    ok, att, org, d = O.scatter(sphere((0, 0, 0), 1, 2, (0.8, 0.8, 0.8), 0.0), (0, 2, 0), rd, (1, 1, 0), (0, 1, 0),
                                True)
    assert ok and tuple(att) == (0.8, 0.8, 0.8) and tuple(org) == (1, 1, 0)
    np.testing.assert_allclose(d, O.unit((1, 1, 0)), atol=1e-12)
    ok, _, org, _ = O.scatter(sphere((0, 0, 0), 1, 2, (0.9, 0.9, 0.9), 0.3), (0, 2, 0), rd, (1, 1, 0), (0, 1, 0),
                              True)
    assert ok and tuple(org) == (1, 1, 0)


def test_metal_high_fuzz_scatters_and_absorbs(O):  # ray/materials_test.go:84-113
    s = sphere((0, 0, 0), 1, 2, (0.7, 0.7, 0.7), 1.5)
    rd = O.unit((1, -1, 0))
    res = {O.scatter(s, (0, 2, 0), rd, (1, 1, 0), (0, 1, 0), True, sample=i)[0] for i in range(50)}
    assert res == {True, False}


@pytest.mark.parametrize(
    "direction,front", [((0, -1, 0), True), ((1, -1, 0), True), ((0, 1, 0), False), ((1, 1, 0), False)]
)
def test_dielectric_scatter(O, direction, front):  # ray/materials_test.go:115-203
    s = sphere((0, 0, 0), 1, 3, (0, 0, 0), 1.5)
    ok, att, org, _ = O.scatter(s, (0, 0, 0), O.unit(direction), (0, 1, 0), (0, 1, 0), front)
    assert ok and tuple(att) == (1, 1, 1) and tuple(org) == (0, 1, 0)


# --------------------------------------------------------- objects_test.go ---
def test_sphere_hit_simple(O):  # ray/objects_test.go:50-72
    s = sphere((0, 0, -1), 0.5)
    hit, rec = O.sphere_hit(s, (0, 0, 0), (0, 0, -1), 1e-6, math.inf)
    assert hit and rec[6] > 0
    assert abs(np.linalg.norm(rec[0:3] - np.array([0, 0, -1])) - 0.5) <= 1e-10


def test_sphere_miss(O):  # ray/objects_test.go:74-89
    assert not O.sphere_hit(sphere((0, 0, -1), 0.5), (0, 0, 0), (2, 0, -1), 1e-6, math.inf)[0]


def test_sphere_hit_normal_and_inside(O):  # ray/objects_test.go:91-133
    hit, rec = O.sphere_hit(sphere((0, 0, 0), 1.0), (2, 0, 0), (-1, 0, 0), 1e-6, math.inf)
    assert hit and rec[7] == 1 and np.linalg.norm(rec[3:6] - np.array([1, 0, 0])) <= 1e-10
    hit, rec = O.sphere_hit(sphere((0, 0, 0), 1.0), (0, 0, 0), (1, 0, 0), 0.0, math.inf)  # Front interval
    assert hit and rec[7] == 0


def test_sphere_hit_interval(O):  # ray/objects_test.go:135-159
    s = sphere((0, 0, -5), 1.0)
    assert O.sphere_hit(s, (0, 0, 0), (0, 0, -1), 0, 10)[0]
    assert not O.sphere_hit(s, (0, 0, 0), (0, 0, -1), 0, 3)[0]
    assert not O.sphere_hit(s, (0, 0, 0), (0, 0, -1), 10, 20)[0]


def test_scene_hit_closest_and_ties(O):  # ray/objects_test.go:161-225
    from oracle.oracle import SPHERE_DTYPE

    sc = np.concatenate([sphere((0, 0, -1), 0.5), sphere((0, 0, -2), 0.5, 2, (0.8, 0.8, 0.8))])
    idx, rec = O.scene_hit(sc, (0, 0, 0), (0, 0, -1), 1e-6, math.inf)
    assert idx == 0 and abs(rec[6] - 0.5) <= 0.1
    assert O.scene_hit(sc[:1], (0, 0, 0), (10, 0, -1), 1e-6, math.inf)[0] == -1
    # identical spheres: strict '<' keeps the earlier object (objects.go:41)
    dup = np.concatenate([sphere((0, 0, -3), 1.0), sphere((0, 0, -3), 1.0)]).astype(SPHERE_DTYPE)
    assert O.scene_hit(dup, (0, 0, 0), (0, 0, -1), 1e-6, math.inf)[0] == 0


def test_ray_color_depth_and_sky(O):  # ray/objects_test.go:227-288
    s = sphere((0, 0, -1), 0.5, 1, (1, 1, 1))
    c, seg = O.ray_color(s, DEFAULT_BG, (0, 0, 0), (0, 0, -1), 0)
    assert tuple(c) == (0, 0, 0) and seg == 0
    c, seg = O.ray_color(s, DEFAULT_BG, (0, 0, 0), (0, 0, -1), 5)
    assert tuple(c) != (0, 0, 0) and 1 <= seg <= 5
    c, _ = O.ray_color(None, DEFAULT_BG, (0, 0, 0), (0, -1, 0), 10)
    assert not c[2] < c[0]  # the Go check: blue never below red
    c, _ = O.ray_color(None, DEFAULT_BG, (0, 0, 0), (0, 1, 0), 10)
    assert tuple(c) == (0.4, 0.65, 1.0)  # zenith = ColorB exactly
    c, _ = O.ray_color(None, np.zeros(6), (0, 0, 0), (0, -1, 0), 10)
    assert tuple(c) == (0, 0, 0)  # zero AmbientLight -> black


@pytest.mark.parametrize("mat,albedo,param", [(1, (0.5, 0.5, 0.5), 0.0), (2, (0.8, 0.8, 0.8), 0.0), (3, (0, 0, 0), 1.5)])
def test_ray_color_materials_in_range(O, mat, albedo, param):  # ray/objects_test.go:290-323
    s = sphere((0, 0, -1), 0.5, mat, albedo, param)
    for i in range(20):
        c, _ = O.ray_color(s, DEFAULT_BG, (0, 0, 0), (0, 0, -1), 5, sample=i)
        assert np.all((c >= 0) & (c <= 1))


def test_ray_color_absorption(O):  # ray/objects_test.go:371-395
    s = sphere((0, 0, -5), 1.0, 2, (0.8, 0.8, 0.8), 5.0)
    for i in range(100):
        c, _ = O.ray_color(s, DEFAULT_BG, (0, 0, 0), (0, 0, -1), 5, sample=i)
        assert np.all((c >= 0) & (c <= 1))


def test_default_scene_materials(O):  # ray/objects_test.go:325-369
    sc = O.default_scene()
    assert set(sc["material"].tolist()) == {1, 2, 3}
    assert sc["param"][3] == 1.0 / 1.5


# ---------------------------------------------------------- camera_test.go ---
def test_camera_defaults(O):  # ray/camera_test.go:37-66
    io, cam = O.camera_initialize(np.zeros(13), 100, 100)
    assert io[10] == 1.0 and io[9] == 90.0 and tuple(io[6:9]) == (0, 1, 0) and tuple(io[3:6]) == (0, 0, -1)
    assert np.any(cam[3:6] != 0) and np.any(cam[6:9] != 0) and np.any(cam[9:12] != 0)


def test_camera_position_equals_lookat(O):  # ray/camera_test.go:15-35
    io, cam = O.camera_initialize(np.array([1, 2, 3, 1, 2, 3, 0, 0, 0, 0, 0, 0, 0.0]), 100, 100)
    assert np.all(np.isfinite(cam)) and np.any(cam[3:6] != 0)


def test_camera_custom_preserved_and_focus_default(O):  # ray/camera_test.go:68-99,164-175
    io, _ = O.camera_initialize(np.array([0, 0, 5, 0, 0, 0, 0, 1, 0, 60.0, 2.0, 0, 0]), 100, 100)
    assert tuple(io[0:3]) == (0, 0, 5) and io[9] == 60.0 and io[10] == 2.0
    io, _ = O.camera_initialize(np.array([0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 2.5, 0, 0]), 100, 100)
    assert io[11] == io[10] == 2.5


def test_get_ray_pinhole_and_dof(O):  # ray/camera_test.go:101-162
    _, cam = O.camera_initialize(np.array([0, 0, 5, 0, 0, 0, 0, 0, 0, 0, 1.0, 0, 0]), 100, 100)
    for args in [(50, 50), (25, 75)]:
        o, _ = O.get_ray(cam, *args)
        assert tuple(o) == (0, 0, 5)
    _, cam = O.camera_initialize(np.array([0, 0, 5, 0, 0, 0, 0, 0, 0, 0, 1.0, 5.0, 0.5]), 100, 100)
    o1, _ = O.get_ray(cam, 50, 50, sample=0)
    o2, _ = O.get_ray(cam, 50, 50, sample=1)
    assert tuple(o1) != tuple(o2)
    for o in (o1, o2):
        assert np.linalg.norm(o - np.array([0, 0, 5])) <= 0.5 / 2


def test_get_ray_pixel_center_and_offset(O):  # ray/camera_test.go:177-243
    _, cam = O.camera_initialize(np.array([0, 0, 0, 0, 0, -1, 0, 0, 0, 90.0, 1.0, 0, 0]), 10, 10)
    o, d = O.get_ray(cam, 5, 5)
    target = cam[3:6] + cam[6:9] * 5 + cam[9:12] * 5
    assert O.near_zero(O.unit(target - cam[0:3]) - O.unit(d))
    _, d2 = O.get_ray(cam, 5, 5, 0.3, 0.2)
    assert tuple(d2) != tuple(d)


def test_go_math_tan_restatement(O):
    """Camera.Initialize's math.Tan (ray/camera.go:93) is Go's Cephes-based
    algorithm, not libm's: the C restatement (oracle; the host copy is checked
    against the same Python restatement by test_abi_cpu.py::
    test_host_go_tan_against_independent_restatement) equals the independent
    Python restatement in tests/golden/make_golden.py bit for bit, stays within
    2 ulp of the correctly rounded tangent, and reproduces Go's own
    tan(Pi/4) = 1 where libm gives 1 - 2^-53."""
    import math
    import struct
    import sys

    from conftest import ROOT

    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    import make_golden

    def bits(v):
        return struct.unpack("<q", struct.pack("<d", v))[0]

    # Go's tan.go prints each coefficient's bit pattern beside its decimal value
    for v, h in zip(make_golden._TAN_P + make_golden._TAN_Q[1:],
                    (0xc0c992d8d24f3f38, 0x413199eca5fc9ddd, 0xc1711fead3299176, 0x40cab8a5eeb36572,
                     0xc13427bc582abc96, 0x4177d98fc2ead8ef, 0xc189afe03cbe5a31)):
        assert bits(v) & (2**64 - 1) == h
    rng = np.random.default_rng(7)
    xs = np.concatenate([rng.uniform(-1.6, 1.6, 20000), rng.uniform(-50, 50, 5000),
                         np.arange(1, 180) * float.fromhex("0x1.1df46a2529d39p-6") / 2])
    for x in xs:
        a, b = O.go_tan(float(x)), make_golden.go_tan(float(x))
        assert a == b
        assert abs(bits(a) - bits(math.tan(float(x)))) <= 2
    quarter = 45 * float.fromhex("0x1.1df46a2529d39p-6")  # vertical_fov 90 (the default) / 2
    assert O.go_tan(quarter) == 1.0 and math.tan(quarter) == 1.0 - 2.0 ** -53
    assert O.go_tan(0.0) == 0.0 and math.isnan(O.go_tan(float("nan"))) and math.isnan(O.go_tan(float("inf")))
