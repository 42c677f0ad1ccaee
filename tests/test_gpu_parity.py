"""HIP megakernel (through the C-ABI) vs the oracle and the golden fixtures.

Parity bar: per-pixel Scene.Hit counts bit-exact (every path decision equal);
linear mean colour within 1e-4 L-inf (BASELINE.json north star), and in
practice within 1e-12: the only arithmetic difference is the attenuation
product order (kernel outer-first, Go recursion inner-first)."""
import ctypes
import os

import numpy as np
import pytest

from conftest import DEFAULT_BG, RICH_SETUP, SKY_EDGE_AA, SKY_EDGE_PINHOLE, load_golden, srgb_boundary_distance

pytestmark = pytest.mark.gpu

TOL = 1e-4        # north-star gate (BASELINE.json)
TIGHT = 1e-12     # observed: product-order ulps only
WORKERS = min(16, os.cpu_count() or 4)


def camera(L, setup, w, h):
    d3 = ctypes.c_double * 3
    cs = L.CameraSetup(d3(*setup[0:3]), d3(*setup[3:6]), d3(*setup[6:9]), *[float(v) for v in setup[9:13]])
    st = L.CameraState()
    L.check(L.lib().tray_camera_initialize(ctypes.byref(cs), w, h, ctypes.byref(st)))
    return st


def bg_struct(L, bg):
    d3 = ctypes.c_double * 3
    return L.Background(d3(*bg[0:3]), d3(*bg[3:6]))


def gpu_render(L, spheres, bg, cam, w, h, spp, depth, radius, seed, **kw):  # kw -> make_params
    p = L.make_params(w, h, depth, spp, radius, seed, **kw)
    return L.render(spheres, bg_struct(L, bg), cam, p, 0, segments=True)


def check(gpu_rgb, gpu_seg, ref_rgb, ref_seg):
    assert gpu_rgb.shape == ref_rgb.shape
    assert np.array_equal(gpu_seg, ref_seg), f"{int((gpu_seg != ref_seg).sum())} pixels took different paths"
    err = float(np.max(np.abs(gpu_rgb - ref_rgb))) if gpu_rgb.size else 0.0
    assert err <= TOL
    assert err <= TIGHT, err


def test_device_present(L):
    assert L.device_count() >= 1


@pytest.mark.parametrize("name", ["rngfree_mirrors", "rngfree_mirrors_deep"])
def test_rngfree_golden(L, name):
    g = load_golden(name)
    st = camera(L, g["camera_setup"], int(g["width"]), int(g["height"]))
    assert np.array_equal(st.as_array(), g["camera"])
    rgb, seg = gpu_render(L, g["spheres"], g["background"], st, int(g["width"]), int(g["height"]), 1,
                          int(g["max_depth"]), 0.5, 77)
    check(rgb, seg, g["rgb"], g["segments"])


CASES = {
    # name: (scene, setup, w, h, spp, depth, radius, seed)
    "default_scene": ("default", np.array([-2, 2, 1, 0, 0, -1, 0, 0, 0, 20.0, 0, 12.0 ** 0.5, 0.1]), 48, 32, 8, 10,
                      0.5, 1),
    "book_seed2_dof": ("rich2", RICH_SETUP, 96, 54, 4, 50, 0.5, 2),
    "book_r1_pinhole": ("rich2", np.r_[RICH_SETUP[:12], 0.0], 80, 45, 1, 50, 0.5, 3),
    "book_radius1": ("rich2", RICH_SETUP, 40, 30, 6, 20, 1.0, 11),
    "book_depth1": ("rich2", RICH_SETUP, 40, 30, 3, 1, 0.5, 4),
    # Go's RenderLines takes a negative RayRadius (InDisc scales by the signed r): the candidate
    # lists must bound the disc by |r|
    "book_negative_radius": ("rich2", RICH_SETUP, 64, 36, 8, 50, -1.5, 12),
    "dense_seed7": ("dense7", RICH_SETUP, 48, 27, 2, 50, 0.5, 7),
    "empty": ("empty", RICH_SETUP, 33, 17, 4, 50, 0.5, 5),
    "seed_zero_and_big": ("rich2", RICH_SETUP, 21, 13, 5, 50, 0.5, 0),
    "seed_high_bits": ("rich2", RICH_SETUP, 21, 13, 5, 50, 0.5, 0xDEADBEEF12345678),
}


def scene_for(O, key):
    return {"default": O.default_scene, "rich2": lambda: O.rich_scene(2), "dense7": lambda: O.rich_scene(7, 22),
            "empty": lambda: O.default_scene()[:0]}[key]()


@pytest.mark.parametrize("case", sorted(CASES))
def test_vs_oracle(L, O, case):
    key, setup, w, h, spp, depth, radius, seed = CASES[case]
    sc = scene_for(O, key)
    st = camera(L, setup, w, h)
    rgb, seg = gpu_render(L, sc, DEFAULT_BG, st, w, h, spp, depth, radius, seed)
    ref, rseg = O.render(sc, DEFAULT_BG, st.as_array(), w, h, spp, depth, radius, seed, workers=WORKERS)
    check(rgb, seg, ref, rseg)


def test_config1_full_size(L, O):
    """BASELINE config 1 (the reference's benchmark/ invocation): 400x225, r=16, d=12, seed 2, full image."""
    sc = O.rich_scene(2)
    st = camera(L, RICH_SETUP, 400, 225)
    rgb, seg = gpu_render(L, sc, DEFAULT_BG, st, 400, 225, 16, 12, 0.5, 2)
    ref, rseg = O.render(sc, DEFAULT_BG, st.as_array(), 400, 225, 16, 12, 0.5, 2, workers=WORKERS)
    check(rgb, seg, ref, rseg)


def test_row_range_and_tiles_are_partition_invariant(L, O):
    sc = O.rich_scene(2)
    w, h = 64, 37
    st = camera(L, RICH_SETUP, w, h)
    full, fseg = gpu_render(L, sc, DEFAULT_BG, st, w, h, 3, 50, 0.5, 8)
    part, pseg = gpu_render(L, sc, DEFAULT_BG, st, w, h, 3, 50, 0.5, 8, y_start=5, y_end=21)  # RenderLines rows
    assert np.array_equal(part, full[5:21]) and np.array_equal(pseg, fseg[5:21])
    from tray_amd import shard

    for world, tile in [(3, 5), (2, 1), (4, 16), (8, 8)]:
        got = np.zeros_like(full)
        for r in range(world):
            out, _ = gpu_render(L, sc, DEFAULT_BG, st, w, h, 3, 50, 0.5, 8, tile_rows=tile, tile_count=world,
                                tile_index=r)
            got[shard.rows_for(h, tile, world, r)] = out
        assert np.array_equal(got, full)
    ref, rseg = O.render(sc, DEFAULT_BG, st.as_array(), w, h, 3, 50, 0.5, 8, workers=WORKERS)
    check(full, fseg, ref, rseg)


def test_output_formats(L, O):
    sc = O.rich_scene(2)
    w, h = 50, 28
    st = camera(L, RICH_SETUP, w, h)
    f64, _ = gpu_render(L, sc, DEFAULT_BG, st, w, h, 4, 50, 0.5, 3)
    f32, _ = gpu_render(L, sc, DEFAULT_BG, st, w, h, 4, 50, 0.5, 3, output=L.OUT_RGB_F32)
    assert f32.dtype == np.float32 and np.array_equal(f32, f64.astype(np.float32))
    u8, _ = gpu_render(L, sc, DEFAULT_BG, st, w, h, 4, 50, 0.5, 3, output=L.OUT_RGBA8)
    # byte output: the fused epilogue's bytes ARE ColorF.ToSRGBA of the linear frame
    assert np.array_equal(u8, O.to_srgba(f64))
    host = np.zeros_like(u8)
    L.check(L.lib().tray_to_srgba(f64.ctypes.data, w * h, host.ctypes.data))
    assert np.array_equal(u8, host)


def srgb_thresholds(O):
    """t[k] = least double whose oracle sRGB byte is >= k (k = 1..255), by bisection
    over the ordered bit patterns of [0, 1] — the table the device encoder counts."""
    lo = np.zeros(255, dtype=np.uint64)
    hi = np.full(255, np.float64(1.0).view(np.uint64), dtype=np.uint64)
    k = np.arange(1, 256)
    while np.any(hi - lo > 1):
        mid = lo + (hi - lo) // np.uint64(2)
        up = O.linear_to_srgb_n(mid.view(np.float64)).astype(int) >= k
        hi = np.where(up, mid, hi)
        lo = np.where(up, lo, mid)
    return hi.view(np.float64)


def test_device_srgb_encoder_bit_exact(L, O):
    """tray_linear_to_srgba_async (the encoder of TRAY_OUT_RGBA8) against the
    oracle's ToSRGBA (ray/vec3.go:173-180) on >= 10^6 channels: random linear
    values, the linear segment, every byte threshold and its +-3 ulp neighbours,
    0, -0, 0.0031308 +- ulps, 1 +- ulp, clamps, infinities and NaN."""
    import torch

    rng = np.random.default_rng(17)
    t = srgb_thresholds(O)
    near = (t.view(np.int64)[:, None] + np.arange(-3, 4)[None, :]).reshape(-1).view(np.float64)
    edge = np.float64(0.0031308)
    special = np.array([0.0, -0.0, 1.0, np.nextafter(1.0, 0), np.nextafter(1.0, 2), edge, np.nextafter(edge, 0),
                        np.nextafter(edge, 1), 0.5, -1.0, 2.0, 1e-300, 5e-324, np.inf, -np.inf, np.nan])
    vals = np.concatenate([rng.random(900_000), rng.random(150_000) * 0.004, rng.random(3000) * 3 - 1, near,
                           special])
    vals = vals[: len(vals) // 3 * 3]
    rgb = torch.as_tensor(vals, device="cuda").reshape(-1, 3).contiguous()
    out = torch.zeros((rgb.shape[0], 4), dtype=torch.uint8, device="cuda")
    L.linear_to_srgba_async(rgb.data_ptr(), rgb.shape[0], out.data_ptr(), 0,
                            torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    assert len(vals) >= 1_000_000
    assert np.array_equal(got[:, :3].reshape(-1), O.linear_to_srgb_n(vals)) and np.all(got[:, 3] == 255)


def test_scene_larger_than_lds(L, O):
    """> 5120 spheres: the kernel reads geometry from global memory instead of LDS."""
    sc = O.rich_scene(5, 40)
    assert len(sc) * 32 > 160 * 1024
    st = camera(L, RICH_SETUP, 24, 14)
    rgb, seg = gpu_render(L, sc, DEFAULT_BG, st, 24, 14, 2, 12, 0.5, 6)
    ref, rseg = O.render(sc, DEFAULT_BG, st.as_array(), 24, 14, 2, 12, 0.5, 6, workers=WORKERS)
    check(rgb, seg, ref, rseg)


def test_ragged_and_tiny_images(L, O):
    sc = O.default_scene()
    for w, h in [(1, 1), (1, 17), (17, 1), (15, 15), (16, 16), (17, 33)]:
        st = camera(L, np.array([-2, 2, 1, 0, 0, -1, 0, 0, 0, 20.0, 0, 3.0, 0.1]), w, h)
        rgb, seg = gpu_render(L, sc, DEFAULT_BG, st, w, h, 3, 10, 0.5, 2)
        ref, rseg = O.render(sc, DEFAULT_BG, st.as_array(), w, h, 3, 10, 0.5, 2)
        check(rgb, seg, ref, rseg)


def test_example_png_sky_rows(L, O):
    rows = load_golden("example_sky_rows")["rows"]
    sc = O.rich_scene(2)
    st = camera(L, RICH_SETUP, 1280, 720)
    u8, seg = gpu_render(L, sc, DEFAULT_BG, st, 1280, 720, 64, 50, 0.5, 2, y_start=0, y_end=49,
                         output=L.OUT_RGBA8)
    assert np.all(seg == 64)
    d = np.abs(u8[..., :3].astype(int) - rows.astype(int))
    assert d.max() <= 1 and (d.max(-1) == 0).mean() >= 0.98
    lin, _ = gpu_render(L, sc, DEFAULT_BG, st, 1280, 720, 64, 50, 0.5, 2, y_start=0, y_end=49)
    assert np.array_equal(O.to_srgba(lin), u8)  # the device encoder's bytes are ToSRGBA of the F64 frame
    assert not np.any((d > 0) & (srgb_boundary_distance(lin) >= SKY_EDGE_AA))
    # pixel-centre pinhole rays: exact bytes except within SKY_EDGE_PINHOLE of a rounding boundary
    setup = RICH_SETUP.copy()
    setup[12] = 0.0
    st0 = camera(L, setup, 1280, 720)
    lin0, seg0 = gpu_render(L, sc, DEFAULT_BG, st0, 1280, 720, 1, 50, 0.5, 2, y_start=0, y_end=49)
    assert np.all(seg0 == 1)
    d0 = np.abs(O.to_srgba(lin0)[..., :3].astype(int) - rows.astype(int))
    near = srgb_boundary_distance(lin0) < SKY_EDGE_PINHOLE
    assert d0.max() <= 1 and near.mean() < 0.03
    assert np.array_equal(d0[~near], np.zeros_like(d0[~near]))


def test_example_png_sky_mask(L, O):
    """example.png's scene-independent sky (tests/golden/make_sky_mask.py: 145,582
    pixels of rows 0..156 no ray of any RichScene's camera footprint can reach a
    sphere from) on the device, under the rules of test_example_png_sky_rows."""
    from conftest import example_sky_mask

    mask, rgb, ymax = example_sky_mask()
    m = mask[:ymax]
    sc = O.rich_scene(2)
    st = camera(L, RICH_SETUP, 1280, 720)
    u8, seg = gpu_render(L, sc, DEFAULT_BG, st, 1280, 720, 64, 50, 0.5, 2, y_start=0, y_end=ymax,
                         output=L.OUT_RGBA8)
    assert np.all(seg[m] == 64)
    d = np.abs(u8[..., :3][m].astype(int) - rgb.astype(int))
    assert d.max() <= 1 and (d.max(-1) == 0).mean() >= 0.98
    lin, _ = gpu_render(L, sc, DEFAULT_BG, st, 1280, 720, 64, 50, 0.5, 2, y_start=0, y_end=ymax)
    assert np.array_equal(O.to_srgba(lin), u8)
    assert not np.any((d > 0) & (srgb_boundary_distance(lin)[m] >= SKY_EDGE_AA))
    setup = RICH_SETUP.copy()
    setup[12] = 0.0
    st0 = camera(L, setup, 1280, 720)
    lin0, seg0 = gpu_render(L, sc, DEFAULT_BG, st0, 1280, 720, 1, 50, 0.5, 2, y_start=0, y_end=ymax)
    assert np.all(seg0[m] == 1)
    d0 = np.abs(O.to_srgba(lin0)[..., :3][m].astype(int) - rgb.astype(int))
    near = srgb_boundary_distance(lin0)[m] < SKY_EDGE_PINHOLE
    assert d0.max() <= 1 and near.mean() < 0.05
    assert np.array_equal(d0[~near], np.zeros_like(d0[~near]))


def test_config2_full_size_properties(L, O):
    """BASELINE config 2 at full size (1280x720, r=64, d=50): determinism, and a
    random spot-check of pixels against the oracle (size-independent parity)."""
    sc = O.rich_scene(2)
    st = camera(L, RICH_SETUP, 1280, 720)
    a, sa = gpu_render(L, sc, DEFAULT_BG, st, 1280, 720, 64, 50, 0.5, 2)
    b, sb = gpu_render(L, sc, DEFAULT_BG, st, 1280, 720, 64, 50, 0.5, 2)
    assert np.array_equal(a, b) and np.array_equal(sa, sb)
    rng = np.random.default_rng(2)
    xs = rng.integers(0, 1280, 96)
    ys = np.concatenate([rng.integers(0, 720, 64), rng.integers(400, 720, 32)])  # extra ground pixels
    ref, rseg = O.render_pixels(sc, DEFAULT_BG, st.as_array(), 1280, 720, 64, 50, 0.5, 2, xs, ys)
    check(a[ys, xs], sa[ys, xs], ref, rseg)
    assert sa.min() >= 64 and sa.max() <= 64 * 50


# ---------------------------------------------------------------- BVH --------
BVH_CASES = {
    # name: (scene, setup, w, h, spp, depth, seed)
    "book_dof": ("rich2", RICH_SETUP, 160, 90, 8, 50, 2),
    "book_pinhole": ("rich2", np.r_[RICH_SETUP[:12], 0.0], 128, 72, 2, 50, 5),
    "dense": ("dense7", RICH_SETUP, 96, 54, 4, 50, 7),
    "default_scene_below_bvh_threshold": ("default", np.array([-2, 2, 1, 0, 0, -1, 0, 0, 0, 20.0, 0, 3.0, 0.1]), 64,
                                          40, 4, 10, 1),
    "top_down": ("rich2", np.array([0.5, 30, 0.25, 0, 0, 0, 0, 0, 1, 40.0, 10.0, 30.0, 0.0]), 96, 96, 4, 50, 3),
    "inside_big_glass": ("rich2", np.array([0.05, 1.1, 0.02, 4, 1, 0, 0, 1, 0, 70.0, 1.0, 4.0, 0.0]), 64, 48, 4, 50, 4),
}


@pytest.mark.parametrize("case", sorted(BVH_CASES))
def test_bvh_equals_linear_scan(L, O, case):
    """The exact-culling BVH must reproduce the reference-order linear scan bit for bit
    (same closest root, ties to the lowest index) on every pixel."""
    key, setup, w, h, spp, depth, seed = BVH_CASES[case]
    sc = scene_for(O, key)
    st = camera(L, setup, w, h)
    bvh, sb = gpu_render(L, sc, DEFAULT_BG, st, w, h, spp, depth, 0.5, seed)
    lin, sl = gpu_render(L, sc, DEFAULT_BG, st, w, h, spp, depth, 0.5, seed, flags=L.FLAG_LINEAR_SCAN)
    assert np.array_equal(sb, sl)
    assert np.array_equal(bvh, lin)


def test_bvh_config1_vs_oracle(L, O):
    """Config 1 at full size through the BVH path (default) against the oracle."""
    sc = O.rich_scene(2)
    st = camera(L, RICH_SETUP, 400, 225)
    rgb, seg = gpu_render(L, sc, DEFAULT_BG, st, 400, 225, 16, 12, 0.5, 2)
    ref, rseg = O.render(sc, DEFAULT_BG, st.as_array(), 400, 225, 16, 12, 0.5, 2, workers=WORKERS)
    check(rgb, seg, ref, rseg)


def test_bvh_adversarial_spheres(L, O):
    """Overlapping, nested, duplicated, tiny and huge spheres: ties and grazing hits."""
    from oracle.oracle import SPHERE_DTYPE

    rng = np.random.default_rng(11)
    n = 300
    s = np.zeros(n, dtype=SPHERE_DTYPE)
    s["center"] = rng.uniform(-3, 3, (n, 3))
    s["radius"] = np.exp(rng.uniform(np.log(1e-3), np.log(2.0), n))
    s["material"] = rng.integers(1, 4, n)
    s["albedo"] = rng.uniform(0.2, 0.95, (n, 3))
    s["param"] = np.where(s["material"] == 3, 1.5, rng.uniform(0, 0.6, n))
    s[50:60] = s[40:50]                     # exact duplicates: tie -> lowest index
    s[60:70] = s[40:50]
    s["radius"][60:70] *= 0.5               # nested
    s[0]["center"], s[0]["radius"] = (0, -5000, 0), 4990.0  # huge ground
    setup = np.array([7.0, 3.0, 6.0, 0, 0, 0, 0, 1, 0, 45.0, 1.0, 9.0, 0.05])
    st = camera(L, setup, 80, 60)
    bvh, sb = gpu_render(L, s, DEFAULT_BG, st, 80, 60, 4, 30, 0.5, 9)
    lin, sl = gpu_render(L, s, DEFAULT_BG, st, 80, 60, 4, 30, 0.5, 9, flags=L.FLAG_LINEAR_SCAN)
    assert np.array_equal(sb, sl) and np.array_equal(bvh, lin)
    ref, rseg = O.render(s, DEFAULT_BG, st.as_array(), 80, 60, 4, 30, 0.5, 9, workers=WORKERS)
    check(bvh, sb, ref, rseg)


def test_bvh_global_spheres(L, O):
    """Spheres kept out of the tree (tested first by every traversal): an enclosing
    dome the camera sits inside, listed last, and the ground, listed first."""
    from oracle.oracle import SPHERE_DTYPE

    base = O.rich_scene(3)
    s = np.zeros(len(base) + 1, dtype=SPHERE_DTYPE)
    s[:len(base)] = base
    s[-1]["center"], s[-1]["radius"], s[-1]["material"] = (0, 0, 0), 5000.0, 1  # dome (hit from inside)
    s[-1]["albedo"] = (0.9, 0.8, 0.7)
    dev = L.DeviceScene(s, bg_struct(L, DEFAULT_BG), 0)
    i = dev.info()
    dev.release()
    assert i.has_bvh == 1 and i.n_global == 2 and i.bound == 5000.0
    for setup, seed in ((RICH_SETUP, 3), (np.array([0.5, 30, 0.25, 0, 0, 0, 0, 0, 1, 40.0, 10.0, 30.0, 0.0]), 4)):
        st = camera(L, setup, 64, 40)
        bvh, sb = gpu_render(L, s, DEFAULT_BG, st, 64, 40, 4, 30, 0.5, seed)
        lin, sl = gpu_render(L, s, DEFAULT_BG, st, 64, 40, 4, 30, 0.5, seed, flags=L.FLAG_LINEAR_SCAN)
        assert np.array_equal(sb, sl) and np.array_equal(bvh, lin)
    ref, rseg = O.render(s, DEFAULT_BG, st.as_array(), 64, 40, 4, 30, 0.5, seed, workers=WORKERS)
    check(bvh, sb, ref, rseg)


def test_stats_counters(L, O):
    import torch

    from tray_amd import ray

    sc = O.rich_scene(2)
    w, h, spp, depth = 64, 36, 4, 50
    st = camera(L, RICH_SETUP, w, h)
    _, rseg = O.render(sc, DEFAULT_BG, st.as_array(), w, h, spp, depth, 0.5, 2, workers=WORKERS)
    dev = L.DeviceScene(sc, bg_struct(L, DEFAULT_BG), 0)
    out = torch.empty((h, w, 3), dtype=torch.float32, device="cuda")
    for flags in (0, L.FLAG_LINEAR_SCAN):
        stats = torch.zeros(3, dtype=torch.int64, device="cuda")
        p = L.make_params(w, h, depth, spp, 0.5, 2, flags=flags)
        dev.render_stats_async(st, p, out.data_ptr(), stats.data_ptr(), torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        seg, sph, box = stats.tolist()
        assert seg == int(rseg.sum())
        if flags:
            assert sph == seg * len(sc) and box == 0
        else:
            assert 0 < sph < seg * len(sc) and box > 0
    dev.release()


def test_scene_info_and_traversal_paths(L, O):
    """The book scene is an LDS-resident 1-sphere-per-leaf BVH; a scene too big
    for LDS traverses from global memory; both equal the linear scan."""
    book = L.DeviceScene(O.rich_scene(2), bg_struct(L, DEFAULT_BG), 0)
    i = book.info()
    assert (i.n_spheres, i.has_bvh, i.leaf_max, i.lds_resident) == (486, 1, 1, 1)
    assert 0 < i.stack_depth <= 48 and i.bound == 2000.0  # ground: y in [-2000, 0]
    assert i.n_global == 1 and i.n_leaves == 485  # the ground sphere is tested before the tree
    big = O.rich_scene(5, 40)
    ib = L.DeviceScene(big, bg_struct(L, DEFAULT_BG), 0).info()
    assert ib.has_bvh == 1 and ib.lds_resident == 0
    tiny = L.DeviceScene(O.default_scene(), bg_struct(L, DEFAULT_BG), 0).info()
    assert tiny.has_bvh == 0
    st = camera(L, RICH_SETUP, 40, 24)
    bvh, sb = gpu_render(L, big, DEFAULT_BG, st, 40, 24, 2, 20, 0.5, 8)
    lin, sl = gpu_render(L, big, DEFAULT_BG, st, 40, 24, 2, 20, 0.5, 8, flags=L.FLAG_LINEAR_SCAN)
    assert np.array_equal(sb, sl) and np.array_equal(bvh, lin)


@pytest.mark.parametrize("seed,half,leaf,mode,resident,slots", [(2, 11, "4", "2", 1, None), (2, 11, "1", "0", 1, None),
                                                                (7, 22, "1", None, 0, None), (7, 22, "4", None, 2, None),
                                                                (7, 22, "4", "1", 2, None), (7, 22, None, None, 2, None),
                                                                (7, 22, None, None, 2, "8"), (2, 11, "1", "2", 1, "8")])
def test_bvh_lds_layouts(L, O, knobs, seed, half, leaf, mode, resident, slots):
    """Every LDS layout of the BVH kernel (1: nodes + geometry; 2: nodes + leaf
    table, geometry from global memory; 0: all global), as chosen per leaf size
    (knob "bvh_leaf") or forced ("bvh_lds_mode"), with the whole stack in LDS
    or most of it in the overflow area, renders the linear scan's bits. The
    dense scene (1,939 spheres) picks 2-sphere leaves, nodes-only."""
    sc = O.rich_scene(seed, half)
    st = camera(L, RICH_SETUP, 48, 27)
    if leaf:
        knobs(bvh_leaf=leaf)
    if mode:
        knobs(bvh_lds_mode=mode)
    if slots:  # stack partly in the global overflow area (the spill kernels)
        knobs(stack_lds_slots=slots)
    info = L.DeviceScene(sc, bg_struct(L, DEFAULT_BG), 0).info()
    assert info.has_bvh == 1 and info.lds_resident == resident
    if leaf is None:
        assert info.leaf_max == 2
    bvh, sb = gpu_render(L, sc, DEFAULT_BG, st, 48, 27, 2, 30, 0.5, seed)
    lin, sl = gpu_render(L, sc, DEFAULT_BG, st, 48, 27, 2, 30, 0.5, seed, flags=L.FLAG_LINEAR_SCAN)
    assert np.array_equal(sb, sl) and np.array_equal(bvh, lin)


def test_bvh_deep_tree(L, O):
    """Spheres shrinking geometrically along a line (SAH peels them one by one):
    a deep tree, bounded by median splits, with a deep traversal stack."""
    from oracle.oracle import SPHERE_DTYPE

    n = 160
    s = np.zeros(n, dtype=SPHERE_DTYPE)
    x = np.cumsum(0.97 ** np.arange(n))
    s["center"][:, 0] = x - x.mean()
    s["center"][:, 1] = 0.3 * np.sin(np.arange(n))
    s["radius"] = 0.45 * 0.97 ** np.arange(n)
    s["material"] = 1 + np.arange(n) % 3
    s["albedo"] = 0.7
    s["param"] = np.where(s["material"] == 3, 1.5, 0.2)
    dev = L.DeviceScene(s, bg_struct(L, DEFAULT_BG), 0)
    assert dev.info().has_bvh == 1
    setup = np.array([0.0, 2.0, 14.0, 0, 0, 0, 0, 1, 0, 60.0, 1.0, 14.0, 0.0])
    st = camera(L, setup, 96, 32)
    bvh, sb = gpu_render(L, s, DEFAULT_BG, st, 96, 32, 2, 30, 0.5, 12)
    lin, sl = gpu_render(L, s, DEFAULT_BG, st, 96, 32, 2, 30, 0.5, 12, flags=L.FLAG_LINEAR_SCAN)
    assert np.array_equal(sb, sl) and np.array_equal(bvh, lin)


def test_launch_bands_are_invisible(L, O, knobs):
    """A frame split into several launch bands (small "band_samples") renders
    the same bits as one band, tiled and untiled."""
    sc = O.rich_scene(2)
    st = camera(L, RICH_SETUP, 72, 41)
    one, s1 = gpu_render(L, sc, DEFAULT_BG, st, 72, 41, 3, 20, 0.5, 4)
    knobs(band_samples=72 * 8 * 3 * 2)  # two 8-row tile rows per band
    many, sm = gpu_render(L, sc, DEFAULT_BG, st, 72, 41, 3, 20, 0.5, 4)
    assert np.array_equal(s1, sm) and np.array_equal(one, many)
    t, stl = gpu_render(L, sc, DEFAULT_BG, st, 72, 41, 3, 20, 0.5, 4, tile_rows=8, tile_count=2, tile_index=1)
    rows = [y for y in range(41) if (y // 8) % 2 == 1]
    assert np.array_equal(t, one[rows]) and np.array_equal(stl, s1[rows])


def test_stack_overflow_area(L, O, knobs):
    """Traversal-stack slots beyond the LDS ones live in a global overflow area:
    forcing the minimum of LDS slots renders the same bits."""
    sc = O.rich_scene(2)
    st = camera(L, RICH_SETUP, 64, 36)
    a, sa = gpu_render(L, sc, DEFAULT_BG, st, 64, 36, 4, 50, 0.5, 3)
    knobs(stack_lds_slots=8)
    b, sb = gpu_render(L, sc, DEFAULT_BG, st, 64, 36, 4, 50, 0.5, 3)
    assert np.array_equal(sa, sb) and np.array_equal(a, b)


def test_progressive_pass_vs_oracle(L, O):
    """tray_params.pass: sample s of a pixel draws RNG sample word pass*r + s
    (include/tray.h). A later pass matches the oracle's render of that pass and
    differs from pass 0."""
    sc = O.rich_scene(2)
    st = camera(L, RICH_SETUP, 64, 36)
    rgb, seg = gpu_render(L, sc, DEFAULT_BG, st, 64, 36, 4, 50, 0.5, 2, pass_=3)
    ref, rseg = O.render(sc, DEFAULT_BG, st.as_array(), 64, 36, 4, 50, 0.5, 2, workers=WORKERS, pass_=3)
    check(rgb, seg, ref, rseg)
    first, _ = gpu_render(L, sc, DEFAULT_BG, st, 64, 36, 4, 50, 0.5, 2)
    assert not np.array_equal(first, rgb)


def _passes(L, dev, st, p, n, dtype, shape):
    import torch

    out = torch.zeros((n,) + shape, dtype=dtype, device="cuda")
    dev.render_passes_async(st, p, n, out.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    return out.cpu().numpy()


@pytest.mark.parametrize("bands", [False, True])
def test_passes_launch_equals_single_passes(L, O, knobs, bands):
    """tray_render_passes_async: n progressive passes in one persistent launch
    are bit-identical to n single-pass renders, in every output format, with one
    or several launch bands and with row tiles."""
    import torch

    sc = O.rich_scene(2)
    w, h, spp = 72, 41, 3
    st = camera(L, RICH_SETUP, w, h)
    if bands:
        knobs(band_samples=72 * 8 * 3 * 3 * 2)  # two 8-row tile rows per band
    dev = L.DeviceScene(sc, bg_struct(L, DEFAULT_BG), 0)
    try:
        for fmt, dtype, ch in [(L.OUT_RGB_F64, torch.float64, 3), (L.OUT_RGB_F32, torch.float32, 3),
                               (L.OUT_RGBA8, torch.uint8, 4)]:
            for tiles in [{}, dict(tile_rows=4, tile_count=3, tile_index=2)]:
                p = L.make_params(w, h, 20, spp, 0.5, 9, output=fmt, pass_=2, **tiles)
                rows = L.params_rows(p)
                frames = _passes(L, dev, st, p, 3, dtype, (rows, w, ch))
                for k in range(3):
                    q = L.make_params(w, h, 20, spp, 0.5, 9, output=fmt, pass_=2 + k, **tiles)
                    one, _ = L.render(sc, bg_struct(L, DEFAULT_BG), st, q, 0)
                    assert np.array_equal(frames[k], one), (fmt, tiles, k)
                assert not np.array_equal(frames[0], frames[1])
    finally:
        dev.release()


def test_passes_argument_checks(L, O):
    import torch

    dev = L.DeviceScene(O.rich_scene(2), bg_struct(L, DEFAULT_BG), 0)
    st = camera(L, RICH_SETUP, 16, 8)
    out = torch.zeros((2, 8, 16, 3), dtype=torch.float64, device="cuda")
    try:
        with pytest.raises(L.TrayError):
            dev.render_passes_async(st, L.make_params(16, 8, 5, 4, 0.5, 1), 0, out.data_ptr())
        with pytest.raises(L.TrayError):
            dev.render_passes_async(st, L.make_params(16, 8, 5, 4, 0.5, 1, pass_=-1), 1, out.data_ptr())
        with pytest.raises(L.TrayError):  # (pass + n) x r beyond the 32-bit sample word
            dev.render_passes_async(st, L.make_params(16, 8, 5, 1 << 30, 0.5, 1, pass_=3), 2, out.data_ptr())
    finally:
        dev.release()


@pytest.mark.parametrize("spp,radius", [(100, 0.5), (128, 0.0), (65, 2.0)])
def test_hollow_glass_and_chunk_straddling_pixels(L, O, spp, radius):
    """RTIOW's hollow glass sphere (a negative-radius inner sphere flips the
    normal, ray/objects.go:100), fuzzed metal, and sample counts whose pixels
    span or straddle 64-sample work chunks; AA disc radius 0 and 2. Linear scan
    and BVH both against the oracle."""
    from oracle.oracle import SPHERE_DTYPE

    s = np.zeros(30, dtype=SPHERE_DTYPE)  # > kBvhMinSpheres: the BVH is built
    rows = [((0, -100.5, -1), 100.0, 1, (0.8, 0.8, 0.0), 0.0),
            ((0, 0, -1.2), 0.5, 1, (0.1, 0.2, 0.5), 0.0),
            ((-1, 0, -1), 0.5, 3, (0, 0, 0), 1.5),
            ((-1, 0, -1), -0.4, 3, (0, 0, 0), 1.5),   # hollow: inner surface, normals inward
            ((1, 0, -1), 0.5, 2, (0.8, 0.6, 0.2), 0.3),
            ((0.3, -0.3, -0.6), 0.15, 2, (0.9, 0.9, 0.9), 0.0)]
    for i, (c, r, m, a, prm) in enumerate(rows):
        s[i]["center"], s[i]["radius"], s[i]["material"], s[i]["albedo"], s[i]["param"] = c, r, m, a, prm
    rng = np.random.default_rng(3)
    s[6:]["center"] = np.c_[rng.uniform(-2, 2, 24), rng.uniform(-0.45, -0.35, 24), rng.uniform(-3, 0, 24)]
    s[6:]["radius"] = rng.uniform(0.03, 0.1, 24)
    s[6:]["material"] = rng.integers(1, 4, 24)
    s[6:]["albedo"] = rng.uniform(0.2, 0.9, (24, 3))
    s[6:]["param"] = np.where(s[6:]["material"] == 3, 1.5, rng.uniform(0, 0.5, 24))
    setup = np.array([-2, 2, 1, 0, 0, -1, 0, 1, 0, 20.0, 0, 3.4, 0.1])
    w, h = 24, 14
    st = camera(L, setup, w, h)
    got, seg = gpu_render(L, s, DEFAULT_BG, st, w, h, spp, 20, radius, 5)
    ref, rseg = O.render(s, DEFAULT_BG, st.as_array(), w, h, spp, 20, radius, 5, workers=WORKERS)
    check(got, seg, ref, rseg)
    lin, sl = gpu_render(L, s, DEFAULT_BG, st, w, h, spp, 20, radius, 5, flags=L.FLAG_LINEAR_SCAN)
    assert np.array_equal(sl, seg) and np.array_equal(lin, got)


@pytest.mark.parametrize("devices", [[0], [0, 0], [0, 0, 0]])
def test_render_devices_equals_single_device(L, O, devices):
    """tray_render_devices (the row split over several devices of one process; on
    one GPU the shards repeat device 0 on separate streams) writes the same rows,
    bytes and segment counts as tray_render, for every output format and for a
    ragged row range."""
    sc = O.rich_scene(2)
    w, h = 70, 43
    st = camera(L, RICH_SETUP, w, h)
    bg = bg_struct(L, DEFAULT_BG)
    for fmt in (L.OUT_RGB_F64, L.OUT_RGB_F32, L.OUT_RGBA8):
        for y0, y1 in ((0, h), (5, 38)):
            p = L.make_params(w, h, 20, 3, 0.5, 6, y_start=y0, y_end=y1, output=fmt)
            one, s1 = L.render(sc, bg, st, p, 0, segments=True)
            many, sm = L.render_devices(sc, bg, st, p, devices, segments=True)
            assert np.array_equal(one, many) and np.array_equal(s1, sm), (fmt, y0, y1)
    with pytest.raises(L.TrayError):  # it tiles rows itself
        L.render_devices(sc, bg, st, L.make_params(w, h, 5, 1, 0.5, 1, tile_rows=2, tile_count=2), devices)


def test_concurrent_synchronous_renders(L, O):
    """The reference's Render is safe to call from several goroutines on distinct
    tracers; so is tray_render from several threads (ctypes releases the GIL):
    calls on one device serialise on its lock and every result equals the
    sequential one, including when the threads alternate between two scenes
    (the device's cached upload is replaced under the lock)."""
    from concurrent.futures import ThreadPoolExecutor

    scenes = [O.rich_scene(2), O.rich_scene(3)]
    w, h = 40, 24
    st = camera(L, RICH_SETUP, w, h)
    bg = bg_struct(L, DEFAULT_BG)
    jobs = [(k % 2, 3 + k) for k in range(12)]

    def run(job):
        sc, seed = job
        p = L.make_params(w, h, 20, 2, 0.5, seed)
        return L.render(scenes[sc], bg, st, p, 0, segments=True)

    seq = [run(j) for j in jobs]
    with ThreadPoolExecutor(6) as ex:
        par = list(ex.map(run, jobs))
    for (a, sa), (b, sb) in zip(seq, par):
        assert np.array_equal(a, b) and np.array_equal(sa, sb)


@pytest.mark.parametrize("chunks", [1, 3, 8, 64])
def test_wave_chunk_reservations_are_invisible(L, O, knobs, chunks):
    """Waves take 1..64 consecutive chunks per work-queue take (knob "wave_chunks",
    forced for the whole launch, past pool ends and into the last partial pool):
    the frames are bit-identical, for progressive passes in one launch (a pixel's
    passes are consecutive items), row tiles and several launch bands."""
    import torch

    sc = O.rich_scene(2)
    w, h, spp = 72, 41, 64
    st = camera(L, RICH_SETUP, w, h)
    dev = L.DeviceScene(sc, bg_struct(L, DEFAULT_BG), 0)
    try:
        base = {}
        for forced in (None, chunks):
            knobs(wave_chunks=forced, band_samples=None)
            for tiles in [{}, dict(tile_rows=4, tile_count=3, tile_index=1)]:
                for band in (None, 72 * 8 * spp * 3 * 2):
                    knobs(band_samples=band)
                    p = L.make_params(w, h, 20, spp, 0.5, 9, output=L.OUT_RGB_F32, pass_=1, **tiles)
                    frames = _passes(L, dev, st, p, 3, torch.float32, (L.params_rows(p), w, 3))
                    key = (str(tiles), band)
                    if forced is None:
                        base[key] = frames
                    else:
                        assert np.array_equal(frames, base[key]), (chunks, tiles, band)
        one, _ = gpu_render(L, sc, DEFAULT_BG, st, w, h, spp, 20, 0.5, 9, output=L.OUT_RGB_F32, pass_=2)
        assert np.array_equal(base[(str({}), None)][1], one)  # frame k of the launch = pass 1 + k rendered alone
    finally:
        dev.release()


def test_config2_full_frame_vs_oracle(L, O):
    """The headline config (C2: 1280x720, r=64, d=50, seed 2) at EVERY one of its
    921,600 pixels against the oracle's render of the same pass (ray/tracer.go:
    120-155 restated): per-pixel Scene.Hit counts bit-exact, the FP64 output
    (tray_render, fixed-point pixel sums) within 1e-12, and frame 0 of a
    16-pass launch in bench.py's timed shape (TRAY_OUT_RGB_F32) within one f32
    rounding of a value inside 1e-12 (bench.frame_parity, the `parity` field of
    the bench line)."""
    import torch

    from bench import frame_parity

    W, H, spp, depth, seed = 1280, 720, 64, 50, 2
    sc = O.rich_scene(2)
    st = camera(L, RICH_SETUP, W, H)
    f64, seg = gpu_render(L, sc, DEFAULT_BG, st, W, H, spp, depth, 0.5, seed)
    dev = L.DeviceScene(sc, bg_struct(L, DEFAULT_BG), 0)
    try:
        out = torch.empty((16, H, W, 3), dtype=torch.float32, device="cuda")
        p = L.make_params(W, H, depth, spp, 0.5, seed, output=L.OUT_RGB_F32)
        assert dev.plan(st, p, 16).acc_slots > 0  # the on-chip sums bench.py times
        dev.render_passes_async(st, p, 16, out.data_ptr(), torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        f32 = out[0].cpu().numpy()
    finally:
        dev.release()
    ref, rseg = O.render(sc, DEFAULT_BG, st.as_array(), W, H, spp, depth, 0.5, seed, workers=WORKERS)
    rec = frame_parity(ref, rseg, f64, seg, f32)
    assert rec["pixels"] == W * H
    assert rec["segments_equal"], rec
    assert rec["linf"] <= TOL and rec["linf"] <= TIGHT, rec
    assert rec["f32_within_one_rounding"] and rec["linf_f32"] <= TOL, rec
    assert rec["ok"]
