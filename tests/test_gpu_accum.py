"""Fixed-point accumulation of a pixel's samples ("Accumulation").

Frames whose rays_per_pixel is a multiple of 64, or 16 or 32 (every benchmark
config) sum each pixel's samples exactly as integers (the colour scaled by 2^k
and rounded, k >= 44, so the mean is within 2^-45 of the exact mean of the FP64
sample colours), on chip when the LDS has room (per 64-sample chunk, or per
pixel-pass of a chunk that holds 64 / r of them), else through the per-sample
buffer. Both mechanisms give the same bits, whatever the
order the samples finish in; against the oracle (Go's FP64 sum in sample order)
the frames stay inside the parity bar of tests/test_gpu_parity.py (paths
bit-exact, colour within 1e-12). Other frames keep the FP64 sum in sample order.
The "acc_slots" knob (include/tray_debug.h) and TRAY_FLAG_ORDERED_SUM are read
at every launch; the process environment is never read."""
import os

import numpy as np
import pytest

from conftest import DEFAULT_BG, RICH_SETUP
from test_gpu_parity import WORKERS, bg_struct, camera, check, gpu_render

pytestmark = pytest.mark.gpu

FIXED_TOL = 2.0 ** -44  # fixed point vs the FP64 sum of the same samples: 2^-45 + the FP64 sum's own rounding


# width/height not multiples of 8: padding pixels in the last tiles (chunks that start no sample)
# r = 16 / 32: a chunk is 4 / 2 pixel-passes (here pixels: one pass), padding and real pixels mixed
@pytest.mark.parametrize("scene,spp", [("rich2", 64), ("rich2", 128), ("dense7", 64), ("rich2", 256), ("dense7", 192),
                                       ("rich2", 16), ("rich2", 32), ("dense7", 16)])
def test_on_chip_equals_sample_buffer_and_oracle(L, O, scene, spp):
    sc = O.rich_scene(2) if scene == "rich2" else O.rich_scene(7, 22)
    w, h = 37, 21
    st = camera(L, RICH_SETUP, w, h)
    base, bseg = gpu_render(L, sc, DEFAULT_BG, st, w, h, spp, 50, 0.5, 5)
    # per-sample buffer with integer resolve; one and two slots per wave (lanes wait for a free slot)
    # (slots 0: the LDS-staged integer resolve when 8 | r, and with resolve_staged=0 the plain one)
    for slots, staged in ((0, 1), (0, 0), (1, 1), (2, 1), (9, 1)):
        with L.debug_knobs(acc_slots=slots, resolve_staged=staged):
            rgb, seg = gpu_render(L, sc, DEFAULT_BG, st, w, h, spp, 50, 0.5, 5)
        assert np.array_equal(seg, bseg), (slots, staged)
        assert np.array_equal(rgb, base), (slots, staged)
    ref, rseg = O.render(sc, DEFAULT_BG, st.as_array(), w, h, spp, 50, 0.5, 5, workers=WORKERS)
    check(base, bseg, ref, rseg)


@pytest.mark.parametrize("spp", [64, 16])
def test_fixed_point_vs_fp64_sum(L, O, spp):
    sc = O.rich_scene(2)
    w, h = 48, 27
    st = camera(L, RICH_SETUP, w, h)
    fixed, fseg = gpu_render(L, sc, DEFAULT_BG, st, w, h, spp, 50, 0.5, 6)
    f64, dseg = gpu_render(L, sc, DEFAULT_BG, st, w, h, spp, 50, 0.5, 6, flags=L.FLAG_ORDERED_SUM)
    assert np.array_equal(fseg, dseg)
    err = float(np.max(np.abs(fixed - f64)))
    assert err <= FIXED_TOL, err
    assert not np.array_equal(fixed, f64)  # the two sums do differ in the last bits somewhere


@pytest.mark.parametrize("spp", [64, 32])
def test_fixed_point_formats_and_linear_scan(L, O, spp):
    sc = O.rich_scene(2)
    w, h = 40, 22
    st = camera(L, RICH_SETUP, w, h)
    f64, seg = gpu_render(L, sc, DEFAULT_BG, st, w, h, spp, 50, 0.5, 3)
    f32, _ = gpu_render(L, sc, DEFAULT_BG, st, w, h, spp, 50, 0.5, 3, output=L.OUT_RGB_F32)
    assert np.array_equal(f32, f64.astype(np.float32))
    u8, _ = gpu_render(L, sc, DEFAULT_BG, st, w, h, spp, 50, 0.5, 3, output=L.OUT_RGBA8)
    assert np.array_equal(u8, O.to_srgba(f64))
    # the linear-scan kernel sums through the per-sample buffer: same bits
    lin, lseg = gpu_render(L, sc, DEFAULT_BG, st, w, h, spp, 50, 0.5, 3, flags=L.FLAG_LINEAR_SCAN)
    assert np.array_equal(lseg, seg) and np.array_equal(lin, f64)


def test_bound_too_large_keeps_fp64_sum(L, O):
    """Albedo 3 at depth 50 bounds the colour at 3^50: no usable scale, so the
    frame is the FP64 sum in sample order (identical to TRAY_FLAG_ORDERED_SUM)."""
    sc = O.rich_scene(2).copy()
    lam = sc["material"] == 1
    sc["albedo"][lam] *= 3.0
    w, h = 24, 14
    st = camera(L, RICH_SETUP, w, h)
    a, sa = gpu_render(L, sc, DEFAULT_BG, st, w, h, 64, 50, 0.5, 2)
    b, sb = gpu_render(L, sc, DEFAULT_BG, st, w, h, 64, 50, 0.5, 2, flags=L.FLAG_ORDERED_SUM)
    assert np.array_equal(sa, sb) and np.array_equal(a, b)
    ref, rseg = O.render(sc, DEFAULT_BG, st.as_array(), w, h, 64, 50, 0.5, 2, workers=WORKERS)
    assert np.array_equal(sa, rseg)
    assert float(np.max(np.abs(a - ref))) <= 1e-12 * max(1.0, float(np.max(np.abs(ref))))


# r = 16 with 3 and 4 passes per launch: a chunk's four pixel-passes straddle pixels
# (3) or are one pixel's passes (4)
@pytest.mark.parametrize("spp,passes", [(128, 3), (16, 3), (16, 4), (32, 5)])
def test_passes_and_tiles_with_chunk_partials(L, O, spp, passes):
    """Several progressive passes in one launch (partials of every pass in one
    buffer), row tiles, and a short launch band: bit-identical to single renders."""
    import torch

    from test_gpu_parity import _passes

    sc = O.rich_scene(2)
    w, h = 37, 19
    st = camera(L, RICH_SETUP, w, h)
    dev = L.DeviceScene(sc, bg_struct(L, DEFAULT_BG), 0)
    try:
        assert dev.plan(st, L.make_params(w, h, 50, spp, 0.5, 4), passes).acc_slots > 0
        for band in (None, 40 * 8 * spp * passes * 2):
            with L.debug_knobs(band_samples=band):
                for tiles in [{}, dict(tile_rows=2, tile_count=3, tile_index=1)]:
                    p = L.make_params(w, h, 50, spp, 0.5, 4, pass_=1, **tiles)
                    rows = L.params_rows(p)
                    frames = _passes(L, dev, st, p, passes, torch.float64, (rows, w, 3))
                    for k in range(passes):
                        q = L.make_params(w, h, 50, spp, 0.5, 4, pass_=1 + k, **tiles)
                        one, _ = L.render(sc, bg_struct(L, DEFAULT_BG), st, q, 0)
                        assert np.array_equal(frames[k], one), (band, tiles, k)
    finally:
        dev.release()


def test_render_plan(L, O):
    """tray_render_plan_get reports which accumulation a render runs: every benchmark
    config sums on chip, C1 (r = 16) one record per pixel-pass, the others one per
    64 samples; r = 8 keeps the FP64 sum in sample order."""
    from bench import CONFIGS
    from tray_amd import ray

    plans = {}
    for c in ("c1", "c2", "c5"):
        _, seed, half, w, h, spp, depth = CONFIGS[c]
        cam = ray.RichSceneCamera()
        cam.Initialize(w, h)
        dev = L.DeviceScene(ray.rich_scene_array(seed, half), ray._background(ray.DefaultBackground()), 0)
        try:
            p = L.make_params(w, h, depth, spp, 0.5, seed, output=L.OUT_RGB_F32)
            plans[c] = dev.plan(cam._state, p, 16).as_dict()
            with L.debug_knobs(acc_slots=0):
                assert dev.plan(cam._state, p, 16).acc_slots == 0
            ordered = L.make_params(w, h, depth, spp, 0.5, seed, output=L.OUT_RGB_F32, flags=L.FLAG_ORDERED_SUM)
            op = dev.plan(cam._state, ordered, 16)
            assert op.fixed_point_shift == 0 and op.acc_slots == 0
            lin = L.make_params(w, h, depth, spp, 0.5, seed, flags=L.FLAG_LINEAR_SCAN)
            assert dev.plan(cam._state, lin, 1).bvh == 0 and dev.plan(cam._state, lin, 1).acc_slots == 0
        finally:
            dev.release()
    for c in ("c1", "c2", "c5"):
        assert plans[c]["fixed_point_shift"] == 46 and plans[c]["acc_slots"] >= 8 and plans[c]["bvh"] == 1, plans[c]
    assert plans["c2"]["lds_layout"] == 1 and plans["c5"]["lds_layout"] == 2
    # C2, 16 frames: one band, one 32-B record per 64 samples
    assert plans["c2"]["buffer_bytes"] == 1280 * 720 * 64 * 16 // 64 * 32
    assert plans["c2"]["lds_bytes"] <= 160 * 1024
    # C1, 16 frames: one band, one 32-B record per pixel-pass (r = 16), padded to 8x8 tiles
    assert plans["c1"]["buffer_bytes"] == 50 * 29 * 64 * 16 * 32 and plans["c1"]["lds_bytes"] <= 160 * 1024
    _, seed, half, w, h, _, depth = CONFIGS["c1"]
    cam = ray.RichSceneCamera()
    cam.Initialize(w, h)
    dev = L.DeviceScene(ray.rich_scene_array(seed, half), ray._background(ray.DefaultBackground()), 0)
    try:
        p8 = dev.plan(cam._state, L.make_params(w, h, depth, 8, 0.5, seed), 16)
        assert p8.fixed_point_shift == 0 and p8.acc_slots == 0
    finally:
        dev.release()


def test_ordered_sum_flag_vs_oracle(L, O):
    """TRAY_FLAG_ORDERED_SUM at r = 64 (where the default is the fixed-point sum):
    Go's FP64 colorSum in sample order (ray/tracer.go:143), so the frame matches the
    oracle to the last bits except the attenuation product order (kernel
    outer-first, Go inner-first): measured 99 % of channels identical."""
    sc = O.rich_scene(2)
    w, h = 44, 25
    st = camera(L, RICH_SETUP, w, h)
    rgb, seg = gpu_render(L, sc, DEFAULT_BG, st, w, h, 64, 50, 0.5, 8, flags=L.FLAG_ORDERED_SUM)
    ref, rseg = O.render(sc, DEFAULT_BG, st.as_array(), w, h, 64, 50, 0.5, 8, workers=WORKERS)
    assert np.array_equal(seg, rseg)
    assert float(np.max(np.abs(rgb - ref))) <= 1e-15
    assert (rgb == ref).mean() >= 0.95
    fixed, _ = gpu_render(L, sc, DEFAULT_BG, st, w, h, 64, 50, 0.5, 8)
    assert (fixed == ref).mean() < (rgb == ref).mean()  # the default is the fixed-point sum


def test_environment_is_ignored(L, O):
    """The product library reads no TRAY_* environment variable (round 3 had
    eleven): setting the old switches changes neither the plan nor the bits."""
    from tray_amd import ray

    sc = O.rich_scene(2)
    w, h = 40, 22
    st = camera(L, RICH_SETUP, w, h)
    base, bseg = gpu_render(L, sc, DEFAULT_BG, st, w, h, 64, 50, 0.5, 3)
    dev = L.DeviceScene(ray.rich_scene_array(2, 11), ray._background(ray.DefaultBackground()), 0)
    p = L.make_params(w, h, 50, 64, 0.5, 3)
    plan0 = dev.plan(st, p, 1).as_dict()
    old = dict(os.environ)
    try:
        os.environ.update({"TRAY_FIXED_POINT": "0", "TRAY_ACC_SLOTS": "0", "TRAY_BAND_SAMPLES": "4096",
                           "TRAY_BVH_LDS_MODE": "0", "TRAY_PRIMARY_CANDIDATES": "0", "TRAY_NODE_DEEP": "1",
                           "TRAY_STACK_LDS_SLOTS": "8", "TRAY_RESOLVE_STAGED": "0", "TRAY_BVH_LEAF": "4"})
        assert dev.plan(st, p, 1).as_dict() == plan0
        rgb, seg = gpu_render(L, sc, DEFAULT_BG, st, w, h, 64, 50, 0.5, 3)
        assert np.array_equal(rgb, base) and np.array_equal(seg, bseg)
    finally:
        os.environ.clear()
        os.environ.update(old)
        dev.release()


@pytest.mark.parametrize("spp", [16, 32])
def test_pixel_pass_sums_in_every_instance(L, O, spp):
    """r = 16 / 32 (one on-chip record per pixel-pass) in the plain, live-progress and
    counting kernel instances: the same frame, and the counted segments equal the
    oracle's Scene.Hit calls."""
    import torch

    sc = O.rich_scene(2)
    w, h, depth = 37, 21, 50
    st = camera(L, RICH_SETUP, w, h)
    p = L.make_params(w, h, depth, spp, 0.5, 7, output=L.OUT_RGB_F32)
    plain, _ = L.render(sc, bg_struct(L, DEFAULT_BG), st, p, 0)
    rows = []
    live, _ = L.render(sc, bg_struct(L, DEFAULT_BG), st, p, 0, progress=rows.append)
    assert np.array_equal(plain, live) and sum(rows) == h
    dev = L.DeviceScene(sc, bg_struct(L, DEFAULT_BG), 0)
    try:
        assert dev.plan(st, p, 1).acc_slots > 0
        out = torch.empty((h, w, 3), dtype=torch.float32, device="cuda")
        stats = torch.zeros(3, dtype=torch.int64, device="cuda")
        dev.render_stats_async(st, p, out.data_ptr(), stats.data_ptr(), torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        assert np.array_equal(out.cpu().numpy(), plain)
    finally:
        dev.release()
    _, rseg = O.render(sc, DEFAULT_BG, st.as_array(), w, h, spp, depth, 0.5, 7, workers=WORKERS)
    assert int(stats[0]) == int(rseg.sum())
