"""Terminal view (main.go:86-131) on the CPU: the
oracle's C restatement of golang.org/x/image/draw's BiLinear and
NearestNeighbor scalers (oracle_scale_*, the checker of the device scaler in
tests/test_gpu_terminal.py) against an independent numpy restatement written
here from the same published algorithm, bit for bit, plus the properties the
scalers must have; and the host-side terminal helpers.

Parity with the Go library itself is UNPINNED: golang.org/x/image v0.35.0
(go.mod:11) is not vendored and the reference holds no fixture of its output."""
import math

import numpy as np
import pytest

from tray_amd import terminal


def rgba(h, w, seed=0, opaque=True):
    rng = np.random.default_rng(seed)
    img = rng.integers(0, 256, (h, w, 4), dtype=np.uint8)
    if opaque:
        img[..., 3] = 255
    else:  # premultiplied: colour <= alpha
        img[..., :3] = np.minimum(img[..., :3], img[..., 3:4])
    return img


def np_taps(dw, sw):
    """newDistrib(BiLinear, dw, sw): per destination pixel, its (coord, weight)
    taps in order and 1 / total weight (x/image/draw scale.go)."""
    scale = sw / dw
    half, arg = 1.0, 1.0
    if scale > 1:
        half, arg = half * scale, 1 / scale
    out = []
    for x in range(dw):
        center = (x + 0.5) * scale - 0.5
        i = max(0, math.floor(center - half))
        j = math.ceil(center + half)
        if j > sw:
            j = max(sw, i)
        taps, total = [], 0.0
        for c in range(i, j):
            t = abs((center - c) * arg)
            if t >= 1.0 or 1 - t == 0:
                continue
            taps.append((c, 1 - t))
            total += 1 - t
        out.append((taps, 1 / total))
    return out


def np_bilinear(src, dw, dh, dst=None):
    """BiLinear.Scale(dst, dst.Bounds(), src, src.Bounds(), draw.Over, nil) with
    Go's op order (float64 sums in tap order, no fused multiply-add)."""
    sh, sw = src.shape[:2]
    hx, vy = np_taps(dw, sw), np_taps(dh, sh)
    s16 = src.astype(np.uint32) * 0x101
    tmp = np.zeros((sh, dw, 4))
    for x, (taps, inv) in enumerate(hx):
        acc = np.zeros((sh, 4))
        for c, w in taps:
            acc = acc + s16[:, c, :].astype(np.float64) * w
        tmp[:, x, :] = acc * (inv / 0xffff)
    out = np.zeros((dh, dw, 4), np.uint8) if dst is None else dst.copy()
    for y, (taps, inv) in enumerate(vy):
        acc = np.zeros((dw, 4))
        for c, w in taps:
            acc = acc + tmp[c] * w
        acc[:, :3] = np.minimum(acc[:, :3], acc[:, 3:4])
        v = np.floor(np.clip(0xffff * (acc * inv) + 0.5, -1.0, 70000.0))  # int32() of a positive float truncates
        f = np.clip(v, 0, 0xffff).astype(np.uint32)
        a1 = (0xffff - f[:, 3:4]) * 0x101
        out[y] = ((out[y].astype(np.uint32) * a1 // 0xffff + f) >> 8).astype(np.uint8)
    return out


def np_nearest(src, dw, dh):
    sh, sw = src.shape[:2]
    sy = (2 * np.arange(dh, dtype=np.uint64) + 1) * sh // (2 * dh)
    sx = (2 * np.arange(dw, dtype=np.uint64) + 1) * sw // (2 * dw)
    return src[sy][:, sx]


SIZES = [((45, 80), (12, 20)), ((90, 160), (45, 80)), ((720, 1280), (48, 160)), ((37, 53), (10, 11)),
         ((64, 64), (64, 13)), ((9, 200), (9, 7)), ((5, 5), (1, 1)), ((33, 47), (32, 46))]


@pytest.mark.parametrize("src_hw,dst_hw", SIZES)
def test_oracle_bilinear_equals_independent_restatement(O, src_hw, dst_hw):
    for opaque in (True, False):
        img = rgba(*src_hw, seed=sum(src_hw), opaque=opaque)
        ref = np_bilinear(img, dst_hw[1], dst_hw[0])
        got = O.scale_rgba(img, dst_hw[1], dst_hw[0], bilinear=True)
        assert np.array_equal(got, ref)
    # Over onto existing contents (main.go draws into a fresh zero image; the scaler blends)
    img = rgba(*src_hw, seed=3, opaque=False)
    dst = rgba(*dst_hw, seed=4)
    assert np.array_equal(O.scale_rgba(img, dst_hw[1], dst_hw[0], True, dst=dst),
                          np_bilinear(img, dst_hw[1], dst_hw[0], dst=dst))


def test_oracle_nearest_equals_independent_restatement(O):
    for (sh, sw), (dh, dw) in [((12, 20), (45, 80)), ((3, 4), (6, 8)), ((7, 9), (50, 33)), ((90, 160), (45, 80))]:
        img = rgba(sh, sw, seed=sh)
        assert np.array_equal(O.scale_rgba(img, dw, dh, bilinear=False), np_nearest(img, dw, dh))


def test_bilinear_properties(O):
    flat = np.full((40, 64, 4), (200, 17, 90, 255), dtype=np.uint8)
    assert np.array_equal(O.scale_rgba(flat, 16, 10, True), flat[:10, :16])  # weights sum to one
    board = np.zeros((8, 8, 4), dtype=np.uint8)
    board[..., 3] = 255
    board[(np.indices((8, 8)).sum(0) % 2) == 0, :3] = 255
    out = O.scale_rgba(board, 4, 4, True)  # 2x shrink: box-like average of black and white
    assert np.all(np.abs(out[..., :3].astype(int) - 127) <= 24) and np.all(out[..., 3] == 255)
    for dw, sw in [(7, 31), (16, 64), (5, 5), (1, 9), (3, 1000)]:
        for taps, inv in np_taps(dw, sw):
            assert taps and abs(sum(w for _, w in taps) * inv - 1) < 1e-12


def test_nearest_grows_by_repetition(O):
    img = rgba(3, 4)
    assert np.array_equal(O.scale_rgba(img, 8, 6, bilinear=False), np.repeat(np.repeat(img, 2, 0), 2, 1))


def test_image_size_follows_main_go():
    assert terminal.image_size(80, 24, 4) == (320, 192)   # main.go:92, two pixel rows per text row
    assert terminal.image_size(80, 24, 0) == (80, 48)     # -s <= 0 means 1 (main.go:63-66)
    assert terminal.image_size(3, 1, 0.5) == (2, 1)       # Go math.Round: halves away from zero


def test_filter_choice_follows_main_go():
    assert terminal.scale_filter(4) == "bilinear"   # supersample > 1: draw.BiLinear (main.go:127)
    assert terminal.scale_filter(0.5) == "nearest"  # < 1: draw.NearestNeighbor (main.go:125)
    assert terminal.scale_filter(1) is None         # == 1: no scaling (main.go:121)


def test_ansi_halfblocks_layout():
    img = rgba(5, 3, 1)[..., :3]
    text = terminal.ansi_halfblocks(img)
    lines = text.split("\n")
    assert len(lines) == 3 and all(line.count("▀") == 3 for line in lines)
    r, g, b = (int(v) for v in img[0, 0])
    assert lines[0].startswith("\x1b[38;2;%d;%d;%dm" % (r, g, b))
    r, g, b = (int(v) for v in img[1, 0])
    assert "\x1b[48;2;%d;%d;%dm" % (r, g, b) in lines[0]
    assert "\x1b[49m" in lines[2]  # odd last row: default background
    # repeated colours are not re-emitted
    flat = np.zeros((2, 5, 3), dtype=np.uint8)
    assert terminal.ansi_halfblocks(flat).count("\x1b[38;2") == 1
