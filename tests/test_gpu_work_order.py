"""Expensive-first work order (DESIGN.md §5 "Work order"): the first launch of a
(camera, rows, rays per pixel, depth) on a launch context counts each 8x8 tile's
Scene.Hit calls in its chunk records; the next launches hand the tiles out most
expensive first. Every pixel's sum is order-free, so the frames must be the
frames of band order bit for bit: one-frame and progressive-pass launches,
r = 64 / 16 (one record per chunk / per pixel-pass), row tiles, several launch
bands, the counting and the ordered launches alike."""
import numpy as np
import pytest

from conftest import DEFAULT_BG, RICH_SETUP
from test_gpu_parity import bg_struct, camera

pytestmark = pytest.mark.gpu


def _frames(L, torch, dev, st, p, passes, launches):
    outs = []
    for k in range(launches):
        q = L.Params.from_buffer_copy(p)
        q.pass_ = p.pass_ + k * passes
        out = torch.empty((passes, L.params_rows(q), p.width, 3), dtype=torch.float64, device="cuda")
        s = torch.cuda.current_stream()
        if passes == 1:
            dev.render_async(st, q, out.data_ptr(), None, s.cuda_stream)
        else:
            dev.render_passes_async(st, q, passes, out.data_ptr(), s.cuda_stream)
        torch.cuda.synchronize()
        outs.append(out.cpu().numpy())
    return outs


@pytest.mark.parametrize("spp,passes,tiles,band", [(64, 1, {}, None), (64, 3, {}, None), (16, 1, {}, None),
                                                    (16, 4, {}, None), (64, 2, dict(tile_rows=1, tile_count=3,
                                                                                    tile_index=2), None),
                                                    (64, 1, {}, 72 * 8 * 64 * 2)])
def test_work_order_is_invisible(L, O, knobs, spp, passes, tiles, band):
    import torch

    sc = O.rich_scene(2)
    w, h = 72, 45
    st = camera(L, RICH_SETUP, w, h)
    p = L.make_params(w, h, 50, spp, 0.5, 9, output=L.OUT_RGB_F64, **tiles)
    if band:
        knobs(band_samples=band)
    dev = L.DeviceScene(sc, bg_struct(L, DEFAULT_BG), 0)
    try:
        assert dev.plan(st, p, passes).acc_slots > 0
        ordered = _frames(L, torch, dev, st, p, passes, 3)  # counting launch, then two ordered ones
    finally:
        dev.release()
    with L.debug_knobs(work_order=0):
        dev = L.DeviceScene(sc, bg_struct(L, DEFAULT_BG), 0)
        try:
            plain = _frames(L, torch, dev, st, p, passes, 3)
        finally:
            dev.release()
    for a, b in zip(ordered, plain):
        assert np.array_equal(a, b)


def test_work_order_follows_the_camera(L, O):
    """A new camera (another order key) recounts: frames of two cameras rendered
    alternately on one context equal their single renders."""
    import torch

    sc = O.rich_scene(2)
    w, h = 64, 40
    st1 = camera(L, RICH_SETUP, w, h)
    setup2 = RICH_SETUP.copy()
    setup2[0] = 11.0
    st2 = camera(L, setup2, w, h)
    p = L.make_params(w, h, 50, 64, 0.5, 4, output=L.OUT_RGB_F64)
    dev = L.DeviceScene(sc, bg_struct(L, DEFAULT_BG), 0)
    try:
        got = []
        for st in (st1, st2, st1, st1, st2):
            got.append(_frames(L, torch, dev, st, p, 1, 1)[0][0])
    finally:
        dev.release()
    want = [L.render(sc, bg_struct(L, DEFAULT_BG), st, p, 0)[0] for st in (st1, st2)]
    for g, st in zip(got, (0, 1, 0, 0, 1)):
        assert np.array_equal(g, want[st])


def test_work_order_with_band_changes(L, O, knobs):
    """One context alternating one-band launches (which count and then use an
    order) with multi-band launches of the same key (which must not use it: a
    band's tiles are numbered within the band): every frame equals band order."""
    import torch

    sc = O.rich_scene(2)
    w, h, spp = 72, 45, 64
    st = camera(L, RICH_SETUP, w, h)
    p = L.make_params(w, h, 50, spp, 0.5, 3, output=L.OUT_RGB_F64)
    knobs(band_samples=9 * 64 * spp * 6)  # one band at 1 pass, three at 3 passes
    seq = (1, 3, 1, 1, 3, 1)

    def run(dev):
        out = []
        for n in seq:
            out += [f for f in _frames(L, torch, dev, st, p, n, 1)[0]]
        return out

    dev = L.DeviceScene(sc, bg_struct(L, DEFAULT_BG), 0)
    try:
        assert dev.plan(st, p, 1).acc_slots > 0
        ordered = run(dev)
    finally:
        dev.release()
    with L.debug_knobs(work_order=0):
        dev = L.DeviceScene(sc, bg_struct(L, DEFAULT_BG), 0)
        try:
            plain = run(dev)
        finally:
            dev.release()
    for a, b in zip(ordered, plain):
        assert np.array_equal(a, b)
