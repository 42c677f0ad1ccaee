"""Randomised parity: random scenes, cameras, backgrounds and render parameters,
whole frames through the C-ABI against the oracle (oracle/tray_oracle.c, the
restatement of ray/tracer.go:120-155 and ray/objects.go:37-109). Same bar as
tests/test_gpu_parity.py: per-pixel Scene.Hit counts bit-exact, colours within
1e-12 (product-order ulps). The scenes mix what the fixed cases keep apart:
hollow (negative-radius) spheres, exact duplicates (index tie-break), nested
and intersecting spheres, tiny and large radii, fuzz above 1, refraction
indices below 1, a ground sphere or none, and cameras inside spheres."""
import numpy as np
import pytest

from test_gpu_parity import TIGHT, WORKERS, bg_struct, camera

pytestmark = pytest.mark.gpu


def random_scene(O, rng, n, ground):
    from oracle.oracle import SPHERE_DTYPE

    s = np.zeros(n, dtype=SPHERE_DTYPE)
    span = rng.uniform(2, 12)
    s["center"] = rng.uniform(-span, span, (n, 3))
    s["radius"] = np.exp(rng.uniform(np.log(2e-3), np.log(0.4 * span), n))
    s["material"] = rng.integers(1, 4, n)
    s["albedo"] = rng.uniform(0.05, 1.0, (n, 3))
    metal = s["material"] == 2
    glass = s["material"] == 3
    s["param"][metal] = rng.choice([0.0, 0.0, 0.3, 1.0, 1.5], metal.sum())
    s["param"][glass] = rng.choice([1.5, 1.33, 2.4, 0.7, 1.0 / 1.5], glass.sum())
    if n >= 8:
        k = n // 8
        s[n - k:] = s[:k]                          # exact duplicates: the lower index must win ties
        s["radius"][n - k // 2:] *= -1.0           # some of them hollow
        s["center"][1] = s["center"][0]            # concentric pair (nested)
        s["radius"][1] = 0.5 * s["radius"][0]
    if ground:
        s[0]["center"], s[0]["radius"], s[0]["material"] = (0, -1000 - span, 0), 1000.0, 1
    return s


def random_setup(rng, spheres, inside):
    tree = spheres[np.abs(spheres["radius"]) < 100]
    span = float(np.abs(tree["center"]).max()) + 1.0 if len(tree) else 5.0
    if inside and len(tree):
        i = int(np.argmax(np.abs(tree["radius"])))
        frm = tree["center"][i] + 0.3 * abs(tree["radius"][i]) * rng.uniform(-1, 1, 3)
    else:
        frm = rng.uniform(-1.5 * span, 1.5 * span, 3)
    at = rng.uniform(-0.3 * span, 0.3 * span, 3)
    vup = [0, 1, 0] if rng.uniform() < 0.8 else list(rng.uniform(-1, 1, 3))
    aperture = 0.0 if rng.uniform() < 0.3 else rng.uniform(0, 1.0)
    return np.r_[frm, at, vup, rng.uniform(10, 120), 1.0, rng.uniform(1, 20), aperture]


N_CASES = 40


@pytest.mark.parametrize("k", range(N_CASES))
def test_random_scene_vs_oracle(L, O, k):
    rng = np.random.default_rng(1000 + k)
    n = [1, 3, 24, 160, 600][k % 5]
    spheres = random_scene(O, rng, n, ground=k % 3 != 2)
    setup = random_setup(rng, spheres, inside=k % 4 == 3)
    w, h = int(rng.integers(17, 65)), int(rng.integers(9, 41))
    spp, depth = int(rng.integers(1, 5)), int(rng.choice([1, 3, 10, 30, 50]))
    radius = float(rng.choice([0.0, 0.5, 1.7]))
    seed = int(rng.integers(0, 2**63))
    bg = np.r_[rng.uniform(0, 1.2, 3), rng.uniform(0, 1.2, 3)]
    st = camera(L, setup, w, h)
    p = L.make_params(w, h, depth, spp, radius, seed)
    rgb, seg = L.render(spheres, bg_struct(L, bg), st, p, 0, segments=True)
    ref, rseg = O.render(spheres, bg, st.as_array(), w, h, spp, depth, radius, seed, workers=WORKERS)
    assert np.array_equal(seg, rseg), f"case {k}: {int((seg != rseg).sum())} pixels took different paths"
    finite = np.isfinite(ref)
    assert np.array_equal(np.isfinite(rgb), finite), k
    err = float(np.max(np.abs(rgb[finite] - ref[finite]))) if finite.any() else 0.0
    assert err <= TIGHT, (k, err)


# Fixed-point pixel sums (64 | r; DESIGN.md §5 "Accumulation") on random scenes:
# backgrounds up to 12 and albedos up to 1.1 move the colour bound, so the scale
# 2^k ranges over its limits and some cases fall back to the FP64 sum in sample
# order (tray_render_plan_get says which). Same bar; the fixed-point frames are
# also compared with the device's own FP64-order frames (TRAY_FLAG_ORDERED_SUM).
N_FIXED = 16


@pytest.mark.parametrize("k", range(N_FIXED))
def test_random_scene_fixed_point_vs_oracle(L, O, k):

    rng = np.random.default_rng(5000 + k)
    n = [3, 24, 160, 600][k % 4]
    spheres = random_scene(O, rng, n, ground=k % 3 != 2)
    if k % 4 == 1:  # albedo above 1: the bound grows with the depth
        spheres["albedo"] *= rng.uniform(1.0, 1.1)
    setup = random_setup(rng, spheres, inside=k % 5 == 4)
    w, h = int(rng.integers(9, 25)), int(rng.integers(5, 17))
    spp, depth = int(rng.choice([64, 128])), int(rng.choice([3, 10, 50]))
    radius = float(rng.choice([0.0, 0.5, 1.7]))
    seed = int(rng.integers(0, 2**63))
    bg = np.r_[rng.uniform(0, 1, 3), rng.uniform(0, 1, 3)] * float(rng.choice([0.3, 1.0, 4.0, 12.0]))
    st = camera(L, setup, w, h)
    p = L.make_params(w, h, depth, spp, radius, seed)
    dev = L.DeviceScene(spheres, bg_struct(L, bg), 0)
    try:
        shift = dev.plan(st, p).fixed_point_shift
    finally:
        dev.release()
    att = max(1.0, float(np.abs(spheres["albedo"][spheres["material"] != 3]).max(initial=0.0)))
    bound = float(np.abs(bg).max()) * att ** depth * 1.001
    assert (shift > 0) == (bound < 2.0 ** (47 - 44)), (k, shift, bound)
    rgb, seg = L.render(spheres, bg_struct(L, bg), st, p, 0, segments=True)
    po = L.Params.from_buffer_copy(p)
    po.flags |= L.FLAG_ORDERED_SUM
    f64, seg2 = L.render(spheres, bg_struct(L, bg), st, po, 0, segments=True)
    ref, rseg = O.render(spheres, bg, st.as_array(), w, h, spp, depth, radius, seed, workers=WORKERS)
    assert np.array_equal(seg, rseg) and np.array_equal(seg2, rseg), k
    finite = np.isfinite(ref)
    assert np.array_equal(np.isfinite(rgb), finite) and np.array_equal(np.isfinite(f64), finite), k
    scale = max(1.0, float(np.abs(ref[finite]).max())) if finite.any() else 1.0
    err = float(np.max(np.abs(rgb[finite] - ref[finite]))) if finite.any() else 0.0
    assert err <= TIGHT * scale, (k, shift, err)
    if shift > 0:
        assert float(np.max(np.abs(rgb[finite] - f64[finite]), initial=0.0)) <= 2.0 ** (-shift + 1), k
    else:
        assert np.array_equal(rgb, f64, equal_nan=True), k


def test_degenerate_camera_nan_in_both_sums(L, O):
    """Up parallel to the view direction: Go's camera basis u = Unit(Cross(Up, w))
    is NaN (ray/camera.go:80), so every colour is NaN; the fixed-point sums
    (r = 64) give NaN in the same channels as the FP64 sum and the oracle."""

    sc = O.rich_scene(2)
    setup = np.array([0.0, 5, 0, 0, 0, 0, 0, 1, 0, 20.0, 10.0, 10.0, 0.1])
    w, h = 12, 8
    st = camera(L, setup, w, h)
    p = L.make_params(w, h, 10, 64, 0.5, 3)
    bg = np.array([1.0, 1.0, 1.0, 0.4, 0.65, 1.0])
    rgb, _ = L.render(sc, bg_struct(L, bg), st, p, 0, segments=True)
    f64, _ = L.render(sc, bg_struct(L, bg), st, L.make_params(w, h, 10, 64, 0.5, 3, flags=L.FLAG_ORDERED_SUM), 0,
                      segments=True)
    ref, _ = O.render(sc, bg, st.as_array(), w, h, 64, 10, 0.5, 3, workers=WORKERS)
    assert np.array_equal(np.isfinite(rgb), np.isfinite(ref)) and np.array_equal(np.isfinite(f64), np.isfinite(ref))
