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
