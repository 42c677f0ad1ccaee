"""The terminal view's device scaler (tray_scale_rgba / tray_scale_rgba_async,
main.go:119-128) against the oracle's restatement of golang.org/x/image/draw's
BiLinear and NearestNeighbor scalers, byte for byte. Parity with the Go library
itself is unpinned (not vendored; no fixture in the reference)."""
import numpy as np
import pytest

from test_terminal_cpu import SIZES, rgba

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("src_hw,dst_hw", SIZES)
def test_device_bilinear_equals_oracle(L, O, src_hw, dst_hw):
    for opaque in (True, False):
        img = rgba(*src_hw, seed=7 + sum(dst_hw), opaque=opaque)
        got = L.scale_rgba(img, dst_hw[1], dst_hw[0], bilinear=True)
        assert np.array_equal(got, O.scale_rgba(img, dst_hw[1], dst_hw[0], bilinear=True))
    img = rgba(*src_hw, seed=5, opaque=False)
    dst = rgba(*dst_hw, seed=6)  # Over blends onto what dst holds
    assert np.array_equal(L.scale_rgba(img, dst_hw[1], dst_hw[0], True, dst=dst),
                          O.scale_rgba(img, dst_hw[1], dst_hw[0], True, dst=dst))


def test_device_nearest_equals_oracle(L, O):
    for (sh, sw), (dh, dw) in [((12, 20), (45, 80)), ((3, 4), (6, 8)), ((7, 9), (50, 33)), ((90, 160), (45, 80))]:
        img = rgba(sh, sw, seed=sh, opaque=False)
        assert np.array_equal(L.scale_rgba(img, dw, dh, bilinear=False), O.scale_rgba(img, dw, dh, bilinear=False))


def test_rendered_frame_to_terminal(L, O):
    """main.go's path: a 4x-supersampled render of the book cover for a 40x12
    terminal (160x96 RGBA8, rendered on the device), scaled to 40x24 on the
    device straight from device memory (tray_scale_rgba_async), equal to the
    oracle's scaling of the same frame; and through tray_amd.terminal."""
    import torch

    from tray_amd import ray, terminal

    W, H = terminal.image_size(40, 12, 4)
    cam = ray.RichSceneCamera()
    cam.Initialize(W, H)
    p = L.make_params(W, H, 20, 4, 0.5, 2, output=L.OUT_RGBA8)
    frame, _ = L.render(ray.rich_scene_array(2), ray._background(ray.DefaultBackground()), cam._state, p)
    ref = O.scale_rgba(frame, 40, 24, bilinear=True)
    assert np.array_equal(terminal.scale_image(frame, 40, 24, 4), ref)
    src = torch.from_numpy(frame).cuda()
    dst = torch.zeros((24, 40, 4), dtype=torch.uint8, device="cuda")
    L.check(L.lib().tray_scale_rgba_async(src.data_ptr(), W, H, dst.data_ptr(), 40, 24, L.SCALE_BILINEAR, 0,
                                          torch.cuda.current_stream().cuda_stream))
    torch.cuda.synchronize()
    assert np.array_equal(dst.cpu().numpy(), ref)
    text = terminal.ansi_halfblocks(ref)
    assert text.count("\n") == 11 and text.count("▀") == 40 * 12


def test_scale_async_stays_in_stream_order(L, O):
    """tray_scale_rgba_async only enqueues: it returns while the work queued
    before it on the same stream has not started (no host sync, no copy outside
    the stream), and the scaled bytes are those of the finished frame. The
    stream is held by a spin kernel of >= 0.1 s ahead of the render, so the check
    does not race the render's ~5 ms."""
    import torch

    from tray_amd import ray

    W, H = 1280, 720
    cam = ray.RichSceneCamera()
    cam.Initialize(W, H)
    dev = L.DeviceScene(ray.rich_scene_array(2), ray._background(ray.DefaultBackground()), 0)
    try:
        stream = torch.cuda.Stream()
        frame = torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda")
        dst = torch.zeros((24, 40, 4), dtype=torch.uint8, device="cuda")
        p = L.make_params(W, H, 50, 64, 0.5, 2, output=L.OUT_RGBA8)
        with torch.cuda.stream(stream):
            torch.cuda._sleep(300_000_000)  # 0.12 s at the shader clock (3 s if it counts the 100-MHz one)
        dev.render_async(cam._state, p, frame.data_ptr(), None, stream.cuda_stream)
        L.check(L.lib().tray_scale_rgba_async(frame.data_ptr(), W, H, dst.data_ptr(), 40, 24, L.SCALE_BILINEAR, 0,
                                              stream.cuda_stream))
        still_running = not stream.query()
        stream.synchronize()
        assert still_running
        assert np.array_equal(dst.cpu().numpy(), O.scale_rgba(frame.cpu().numpy(), 40, 24, bilinear=True))
    finally:
        dev.release()


def test_scale_after_shutdown(L, O):
    """tray_shutdown frees the scaler's pinned staging buffers too; the next
    scale allocates new ones and gives the same bytes."""
    img = rgba(45, 80, seed=11, opaque=False)
    ref = O.scale_rgba(img, 30, 17, bilinear=True)
    assert np.array_equal(L.scale_rgba(img, 30, 17, bilinear=True), ref)
    L.check(L.lib().tray_shutdown())
    assert np.array_equal(L.scale_rgba(img, 30, 17, bilinear=True), ref)


def test_scale_beside_shutdown_threads(L, O):
    """tray_shutdown frees idle staging buffers while another thread scales:
    entries keep their addresses (a list), so a scale holding one outside the
    lock never sees it moved or freed. Every scaled image is right."""
    import threading

    img = rgba(45, 80, seed=13, opaque=False)
    ref = O.scale_rgba(img, 30, 17, bilinear=True)
    stop = threading.Event()
    bad, errors = [], []

    def scaler():
        try:
            for _ in range(60):
                if not np.array_equal(L.scale_rgba(img, 30, 17, bilinear=True), ref):
                    bad.append(1)
        except BaseException as e:  # noqa: BLE001 - reported below
            errors.append(e)
        finally:
            stop.set()

    def closer():
        try:
            while not stop.is_set():
                L.check(L.lib().tray_shutdown())
        except BaseException as e:  # noqa: BLE001
            errors.append(e)

    ts = [threading.Thread(target=scaler), threading.Thread(target=scaler), threading.Thread(target=closer)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=100)
    assert not errors and not bad
