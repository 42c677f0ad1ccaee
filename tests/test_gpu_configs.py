"""BASELINE.json configs C2-C5 rendered at FULL size on the device, checked
against the oracle pixel by pixel where the oracle can afford it.

Each config's whole frame goes through tray_render_async (with its launch
bands: C3, C4 and C5 need several 2^31-sample bands); >= 256
pixels per config are re-rendered by the oracle (ray/tracer.go:120-155
restated): per-pixel Scene.Hit counts bit-exact, colour within 1e-12 (north-star
gate 1e-4). The picks are biased to where paths are long (glass and metal: the
most Scene.Hit calls), to ground pixels, and to the rows either side of every
launch-band boundary. C4 (the 8-GPU config) is also rendered as eight
interleaved 1-row shards of a row band and compared bit for bit with the
unsharded rows."""
import os
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

from conftest import DEFAULT_BG

pytestmark = pytest.mark.gpu

TOL, TIGHT = 1e-4, 1e-12
WORKERS = min(16, os.cpu_count() or 4)
MAX_BAND_SAMPLES = 1 << 30  # tray_kernel.hpp kMaxBandSamples (per-sample buffer)
MAX_BAND_SAMPLES_ACC = 1 << 31  # kMaxBandSamplesAcc (on-chip chunk sums: the configs here)


def band_rows(W, spp, limit=MAX_BAND_SAMPLES_ACC):
    """Rows per launch band (launch_render: bands of 8-row tile rows, <= limit samples)."""
    return 8 * max(1, limit // (((W + 7) // 8) * 64 * spp))


def render_frame(L, ray, config):
    import torch

    from bench import CONFIGS

    _, seed, half, W, H, spp, depth = CONFIGS[config]
    spheres = ray.rich_scene_array(seed, half)
    cam = ray.RichSceneCamera()
    cam.Initialize(W, H)
    dev = L.DeviceScene(spheres, ray._background(ray.DefaultBackground()), 0)
    try:
        out = torch.empty((H, W, 3), dtype=torch.float64, device="cuda")
        seg = torch.empty((H, W), dtype=torch.int32, device="cuda")
        p = L.make_params(W, H, depth, spp, 0.5, seed)
        dev.render_async(cam._state, p, out.data_ptr(), seg.data_ptr(), torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
    finally:
        dev.release()
    return spheres, cam, (seed, W, H, spp, depth), out, seg


def picks(seg_host, W, H, spp, rng, n_random=96, n_long=64, n_ground=64, n_band=48):
    """Pixel picks: random, longest paths, ground rows, launch-band boundary rows."""
    xs = [rng.integers(0, W, n_random)]
    ys = [rng.integers(0, H, n_random)]
    flat = np.argsort(seg_host.reshape(-1), kind="stable")[::-1][: 50 * n_long]
    chosen = rng.choice(flat, n_long, replace=False)
    xs.append(chosen % W), ys.append(chosen // W)
    xs.append(rng.integers(0, W, n_ground)), ys.append(rng.integers(int(0.6 * H), H, n_ground))
    # the rows either side of every band boundary, with and without chunk records
    edges = sorted({y for lim in (MAX_BAND_SAMPLES_ACC, MAX_BAND_SAMPLES)
                    for b in (band_rows(W, spp, lim),) for k in range(b, H, b) for y in (k - 1, k)}) or [0, H - 1]
    ys.append(rng.choice(np.array(edges), n_band)), xs.append(rng.integers(0, W, n_band))
    return np.concatenate(xs).astype(np.int32), np.concatenate(ys).astype(np.int32)


def oracle_pixels(O, spheres, cam, cfg, xs, ys):
    seed, W, H, spp, depth = cfg
    parts = np.array_split(np.arange(len(xs)), WORKERS)
    with ThreadPoolExecutor(WORKERS) as ex:  # ctypes releases the GIL
        res = list(ex.map(lambda ix: O.render_pixels(spheres, DEFAULT_BG, cam._state.as_array(), W, H, spp, depth,
                                                     0.5, seed, xs[ix], ys[ix]), parts))
    return np.concatenate([r[0] for r in res]), np.concatenate([r[1] for r in res])


@pytest.mark.parametrize("config", ["c2", "c3", "c4", "c5"])
def test_config_full_frame_vs_oracle(L, O, config):
    from tray_amd import ray

    spheres, cam, cfg, out, seg = render_frame(L, ray, config)
    seed, W, H, spp, depth = cfg
    seg_host = seg.cpu().numpy().astype(np.uint32)
    assert seg_host.min() >= spp and seg_host.max() <= spp * depth  # every sample traced, none past MaxDepth
    assert not np.isnan(out.cpu().numpy()).any()
    xs, ys = picks(seg_host, W, H, spp, np.random.default_rng({"c2": 2, "c3": 3, "c4": 4, "c5": 5}[config]))
    assert len(xs) >= 256
    ref, rseg = oracle_pixels(O, spheres, cam, cfg, xs, ys)
    got = out.cpu().numpy()[ys, xs]
    assert np.array_equal(seg_host[ys, xs], rseg), f"{int((seg_host[ys, xs] != rseg).sum())} pixels differ in paths"
    err = float(np.abs(got - ref).max())
    assert err <= TOL and err <= TIGHT, err


def test_config4_row_shards_bit_identical(L, knobs):
    """C4 as the 8-GPU bench splits it (1-row interleaved tiles, tile k -> rank k
    mod 8), rendered shard by shard on one device for a 64-row window, equals the
    unsharded rows bit for bit; the unsharded render is split into launch bands
    of 32 rows (band_samples knob: C4's own bands, 2^31 samples, are 544 rows)."""
    import torch

    from bench import CONFIGS
    from tray_amd import ray, shard

    _, seed, half, W, H, spp, depth = CONFIGS["c4"]
    spheres = ray.rich_scene_array(seed, half)
    cam = ray.RichSceneCamera()
    cam.Initialize(W, H)
    dev = L.DeviceScene(spheres, ray._background(ray.DefaultBackground()), 0)
    y0, y1 = 1064, 1128
    stream = torch.cuda.current_stream().cuda_stream
    try:
        whole = torch.empty((y1 - y0, W, 3), dtype=torch.float64, device="cuda")
        knobs(band_samples=4 * ((W + 7) // 8) * 64 * spp)  # 4 tile rows per band: a boundary at row y0 + 32
        dev.render_async(cam._state, L.make_params(W, H, depth, spp, 0.5, seed, y_start=y0, y_end=y1),
                         whole.data_ptr(), None, stream)
        torch.cuda.synchronize()
        L.clear_debug_knobs()
        got = torch.zeros_like(whole)
        for k in range(8):
            p = L.make_params(W, H, depth, spp, 0.5, seed, y_start=y0, y_end=y1, tile_rows=1, tile_count=8,
                              tile_index=k)
            part = torch.empty((L.params_rows(p), W, 3), dtype=torch.float64, device="cuda")
            dev.render_async(cam._state, p, part.data_ptr(), None, stream)
            torch.cuda.synchronize()
            got[torch.as_tensor(shard.rows_for(H, 1, 8, k, y0, y1) - y0, device="cuda", dtype=torch.long)] = part
        torch.cuda.synchronize()
        assert torch.equal(got, whole)
    finally:
        dev.release()
