"""Terminal sink of the reference's interactive binary (main.go:86-131): render at
`supersample` x the terminal's cell grid (two pixel rows per text row), scale
down bilinearly, draw with upper-half-block characters in 24-bit colour.

Host code, not on the hot path. Parity unpinned: the
scaler restates the published algorithm of golang.org/x/image/draw's
`BiLinear.Scale` (a separable triangle-kernel filter whose support widens by
the downscale factor, weights normalised per output pixel) and the drawing
restates fortio.org/terminal/ansipixels' half-block output; neither library is
present in the reference tree, and the reference's tests hold no fixture for
either, so only the properties in tests/test_terminal_cpu.py are checked.
"""
from __future__ import annotations

import math
import os

import numpy as np


def _weights(dw: int, sw: int, nearest: bool) -> np.ndarray:
    """[dw, sw] contribution matrix, rows normalised (x/image/draw newDistrib:
    center = (x + 0.5)·scale − 0.5, support 1 widened to `scale` when shrinking)."""
    scale = sw / dw
    w = np.zeros((dw, sw), dtype=np.float64)
    if nearest:  # NearestNeighbor.Scale: source pixel floor((x + 0.5)·scale)
        w[np.arange(dw), np.minimum(((np.arange(dw) + 0.5) * scale).astype(np.int64), sw - 1)] = 1.0
        return w
    half, arg_scale = 1.0, 1.0
    if scale > 1:
        half, arg_scale = scale, 1.0 / scale
    for x in range(dw):
        center = (x + 0.5) * scale - 0.5
        i = max(0, math.floor(center - half))
        j = min(sw, math.ceil(center + half))
        if j < i:
            j = i
        ks = np.arange(i, j)
        r = 1.0 - np.abs((center - ks) * arg_scale)  # triangle kernel, zero outside |t| < 1
        r = np.where(r > 0, r, 0.0)
        tot = r.sum()
        if tot > 0:
            w[x, i:j] = r / tot
        else:  # no tap inside the support: nearest source pixel
            w[x, min(sw - 1, max(0, math.floor(center + 0.5)))] = 1.0
    return w


def scale_image(img: np.ndarray, dw: int, dh: int) -> np.ndarray:
    """Scale an [H, W, 4] uint8 RGBA image to [dh, dw, 4]: bilinear when
    shrinking or equal (main.go:124-126 BiLinear), nearest when growing (:122)."""
    sh, sw = img.shape[:2]
    if (sh, sw) == (dh, dw):
        return img.copy()
    nearest = dw > sw or dh > sh
    wx, wy = _weights(dw, sw, nearest), _weights(dh, sh, nearest)
    src = img.astype(np.float64) * 257.0  # 16-bit channels, as image/color's RGBA()
    tmp = np.einsum("xs,hsc->hxc", wx, src)
    out = np.einsum("ys,sxc->yxc", wy, tmp)
    return (np.clip(np.floor(out + 0.5), 0, 65535).astype(np.uint32) >> 8).astype(np.uint8)


def ansi_halfblocks(img: np.ndarray) -> str:
    """Half-block text for an [H, W, 3|4] uint8 image: each text cell is '▀'
    with the upper pixel as foreground and the lower one as background
    (ansipixels' truecolor image mode); colour codes are emitted only when they
    change, and an odd last row is drawn over the default background."""
    h, w = img.shape[:2]
    out = []
    for y in range(0, h, 2):
        fg_prev = bg_prev = ()  # () matches no colour, nor the default background (None)
        line = []
        for x in range(w):
            fg = tuple(int(v) for v in img[y, x, :3])
            bg = tuple(int(v) for v in img[y + 1, x, :3]) if y + 1 < h else None
            if fg != fg_prev:
                line.append("\x1b[38;2;%d;%d;%dm" % fg)
                fg_prev = fg
            if bg != bg_prev:
                line.append("\x1b[49m" if bg is None else "\x1b[48;2;%d;%d;%dm" % bg)
                bg_prev = bg
            line.append("▀")
        line.append("\x1b[0m")
        out.append("".join(line))
    return "\n".join(out)


def terminal_size() -> tuple[int, int]:
    """(columns, rows) of stdout's terminal, (80, 24) when it is not one
    (ansipixels.NonRawTerminalSize)."""
    try:
        s = os.get_terminal_size()
        return s.columns, s.lines
    except OSError:
        return 80, 24


def image_size(cols: int, rows: int, supersample: float) -> tuple[int, int]:
    """Render size for a cols x rows terminal (main.go:88): two pixel rows per
    text row, times the supersampling factor (<= 0 means 1, main.go:63-66)."""
    s = supersample if supersample > 0 else 1.0
    return math.floor(s * cols + 0.5), math.floor(s * rows * 2 + 0.5)  # Go math.Round
