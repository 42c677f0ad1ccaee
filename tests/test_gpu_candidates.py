"""Primary-ray candidate lists (launch_cand_build, tray_kernel.hip) against the
plain BVH traversal: camera rays tested only against their pixel's candidate
spheres must reproduce every Scene.Hit of the traversal bit for bit (per-pixel
segment counts and colours identical), for lenses open and closed, one and many
samples per pixel, wide and narrow fields of view, cameras inside spheres, row
ranges and tilings, and the cached list must follow camera and row changes.
The traversal itself is pinned to the reference-order linear scan by
tests/test_gpu_parity.py (test_bvh_equals_linear_scan)."""
import numpy as np
import pytest

from conftest import DEFAULT_BG, RICH_SETUP
from test_gpu_parity import bg_struct, camera

pytestmark = pytest.mark.gpu


def candidates(on: bool):
    from tray_amd import _lib

    return _lib.debug_knobs(primary_candidates=1 if on else 0)


def both(L, spheres, setup, w, h, spp, depth, radius, seed, **kw):
    st = camera(L, setup, w, h)
    p = L.make_params(w, h, depth, spp, radius, seed, **kw)
    with candidates(False):
        ref = L.render(spheres, bg_struct(L, DEFAULT_BG), st, p, 0, segments=True)
    with candidates(True):
        got = L.render(spheres, bg_struct(L, DEFAULT_BG), st, p, 0, segments=True)
    return got, ref


def adversarial(O):
    from oracle.oracle import SPHERE_DTYPE

    rng = np.random.default_rng(5)
    n = 240
    s = np.zeros(n, dtype=SPHERE_DTYPE)
    s["center"] = rng.uniform(-4, 4, (n, 3))
    s["radius"] = np.exp(rng.uniform(np.log(1e-3), np.log(1.5), n))
    s["material"] = rng.integers(1, 4, n)
    s["albedo"] = rng.uniform(0.2, 0.95, (n, 3))
    s["param"] = np.where(s["material"] == 3, 1.5, rng.uniform(0, 0.5, n))
    s[40:50] = s[20:30]                               # duplicates: tie -> lowest index
    s["radius"][45:50] *= -1.0                         # hollow (negative radius) copies
    s[0]["center"], s[0]["radius"] = (0, -3000, 0), 2995.0  # ground
    s[1]["center"], s[1]["radius"], s[1]["material"], s[1]["param"] = (6.0, 2.5, 5.0), 2.0, 3, 1.5  # holds the camera
    return s


CASES = {
    # name: (scene, setup, w, h, spp, depth, radius, seed, extra params)
    "book_dof_r8": ("rich2", RICH_SETUP, 160, 90, 8, 50, 0.5, 2, {}),
    "book_pinhole_r1": ("rich2", np.r_[RICH_SETUP[:12], 0.0], 160, 90, 1, 50, 0.5, 3, {}),
    "book_pinhole_r4": ("rich2", np.r_[RICH_SETUP[:12], 0.0], 120, 68, 4, 20, 0.5, 4, {}),
    "book_dof_r1": ("rich2", RICH_SETUP, 120, 68, 1, 20, 0.5, 6, {}),
    "book_radius2": ("rich2", RICH_SETUP, 96, 54, 4, 20, 2.0, 11, {}),
    "book_negative_radius": ("rich2", RICH_SETUP, 96, 54, 16, 20, -2.0, 13, {}),
    "book_wide_fov": ("rich2", np.r_[RICH_SETUP[:9], 120.0, RICH_SETUP[10:]], 128, 72, 4, 20, 0.5, 12, {}),
    "book_narrow_fov": ("rich2", np.r_[RICH_SETUP[:9], 4.0, RICH_SETUP[10:]], 128, 72, 4, 20, 0.5, 13, {}),
    "book_top_down": ("rich2", np.array([0.5, 15, 0.2, 0, 0, 0, 0, 0, 1, 60.0, 1.0, 15.0, 0.3]), 96, 96, 4, 20,
                      0.5, 14, {}),
    "book_big_aperture": ("rich2", np.r_[RICH_SETUP[:12], 2.0], 96, 54, 4, 20, 0.5, 15, {}),
    "dense7": ("dense7", RICH_SETUP, 192, 108, 4, 50, 0.5, 7, {}),
    "adversarial_inside": ("adv", np.array([6.0, 2.5, 5.0, 0, 0, 0, 0, 1, 0, 60.0, 1.0, 6.0, 0.1]), 96, 72, 4, 30,
                           0.5, 9, {}),
    "adversarial_outside": ("adv", np.array([11.0, 4.0, 9.0, 0, 0, 0, 0, 1, 0, 50.0, 1.0, 14.0, 0.2]), 96, 72, 4,
                            30, 0.5, 10, {}),
    "row_range": ("rich2", RICH_SETUP, 128, 72, 4, 50, 0.5, 16, {"y_start": 17, "y_end": 55}),
    "tiles_3_of_4": ("rich2", RICH_SETUP, 128, 72, 4, 50, 0.5, 17, {"tile_rows": 1, "tile_count": 4, "tile_index": 3}),
}


def scene(O, key):
    return {"rich2": lambda: O.rich_scene(2), "dense7": lambda: O.rich_scene(7, 22),
            "adv": lambda: adversarial(O)}[key]()


@pytest.mark.parametrize("case", sorted(CASES))
def test_candidates_equal_traversal(L, O, case):
    key, setup, w, h, spp, depth, radius, seed, extra = CASES[case]
    (rgb, seg), (ref, rseg) = both(L, scene(O, key), setup, w, h, spp, depth, radius, seed, **extra)
    assert np.array_equal(seg, rseg), f"{int((seg != rseg).sum())} pixels took different paths"
    assert np.array_equal(rgb, ref)


def test_candidates_equal_traversal_config2_full_frame(L, O):
    """BASELINE config 2 (1280x720, r=64, d=50) over the whole frame."""
    (rgb, seg), (ref, rseg) = both(L, O.rich_scene(2), RICH_SETUP, 1280, 720, 64, 50, 0.5, 2)
    assert np.array_equal(seg, rseg)
    assert np.array_equal(rgb, ref)


def _stats(L, sc, st, p):
    import torch

    out = torch.empty((L.params_rows(p), p.width, 3), dtype=torch.float32, device="cuda")
    stats = torch.zeros(3, dtype=torch.int64, device="cuda")
    sc.render_stats_async(st, p, out.data_ptr(), stats.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    return [int(v) for v in stats.tolist()], out.cpu().numpy()


def test_candidates_replace_primary_traversal(L, O):
    """The path is really taken: same segments and frame, far fewer box tests
    (camera rays no longer traverse), sphere tests of the same order."""
    sc = L.DeviceScene(O.rich_scene(2), bg_struct(L, DEFAULT_BG))
    st = camera(L, RICH_SETUP, 320, 180)
    p = L.make_params(320, 180, 50, 16, 0.5, 2)
    with candidates(False):
        (seg0, sph0, box0), img0 = _stats(L, sc, st, p)
    with candidates(True):
        (seg1, sph1, box1), img1 = _stats(L, sc, st, p)
    sc.release()
    assert seg1 == seg0 and np.array_equal(img0, img1)
    samples = 320 * 180 * 16
    assert box0 - box1 > 10 * samples, (box0, box1)    # ~17 box tests per camera ray saved
    assert abs(sph1 - sph0) < 0.5 * samples, (sph0, sph1)


def test_candidate_cache_follows_camera_and_rows(L, O):
    """One DeviceScene rendered with camera A, camera B, then A with another row
    set: each equals a fresh render without candidates (the cached list is
    rebuilt whenever the camera or the rows change)."""
    import torch

    spheres = O.rich_scene(2)
    sc = L.DeviceScene(spheres, bg_struct(L, DEFAULT_BG))
    setups = [RICH_SETUP, np.r_[[6.0, 3.0, -7.0], RICH_SETUP[3:]], RICH_SETUP]
    extras = [{}, {}, {"y_start": 10, "y_end": 40}]
    w, h = 96, 54
    for setup, extra in zip(setups, extras):
        st = camera(L, setup, w, h)
        p = L.make_params(w, h, 30, 4, 0.5, 21, output=L.OUT_RGB_F64, **extra)
        rows = L.params_rows(p)
        out = torch.empty((rows, w, 3), dtype=torch.float64, device="cuda")
        with candidates(True):
            sc.render_async(st, p, out.data_ptr(), None, torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        with candidates(False):
            ref, _ = L.render(spheres, bg_struct(L, DEFAULT_BG), st, p, 0)
        assert np.array_equal(out.cpu().numpy(), ref)
    sc.release()


def test_candidates_equal_traversal_random_cameras(L, O):
    """24 random cameras (position inside and outside the spheres, any target,
    field of view 5-150 degrees, aperture 0-3, focus 0.5-30, AA radius -3..3: Go takes a signed RayRadius) on the
    adversarial scene and the dense scene: identical frames with and without
    candidate lists."""
    rng = np.random.default_rng(2024)
    scenes = [adversarial(O), O.rich_scene(7, 22)]
    for k in range(24):
        sc = scenes[k % 2]
        span = 8.0 if k % 2 == 0 else 25.0
        frm = rng.uniform(-span, span, 3)
        frm[1] = abs(frm[1]) + 0.5
        at = rng.uniform(-span / 2, span / 2, 3)
        at[1] = rng.uniform(0, 2)
        vfov = rng.uniform(5, 150)
        aperture = 0.0 if k % 4 == 1 else rng.uniform(0, 3)
        focus = rng.uniform(0.5, 30)
        setup = np.r_[frm, at, [0, 1, 0], vfov, 1.0, focus, aperture]
        spp = [1, 2, 4][k % 3]
        radius = rng.uniform(-3, 3)
        (rgb, seg), (ref, rseg) = both(L, sc, setup, 48, 32, spp, 8, radius, 100 + k)
        assert np.array_equal(seg, rseg), (k, setup, spp, radius)
        assert np.array_equal(rgb, ref, equal_nan=True), (k, setup, spp, radius)
