"""Terminal sink of the reference's interactive binary (main.go:86-131): render at
`supersample` x the terminal's cell grid (two pixel rows per text row), scale to
the terminal with golang.org/x/image/draw's scalers (BiLinear when
supersampling, NearestNeighbor below 1, none at 1: main.go:119-128), draw with
upper-half-block characters in 24-bit colour.

Not on the hot path. The scaling runs on the device
(tray_scale_rgba, tray_amd/csrc/tray_scale.hip), byte-identical to the oracle's
restatement of the draw package's published algorithm; parity with the Go
library itself is unpinned (golang.org/x/image and fortio.org/terminal are not
vendored, and the reference holds no fixture of either).
"""
from __future__ import annotations

import math
import os

import numpy as np

from . import _lib


def scale_filter(supersample: float):
    """main.go:121-128: the scaler for a supersampling factor ('bilinear',
    'nearest', or None when the image already has the terminal's size)."""
    if supersample == 1:
        return None
    return "nearest" if supersample < 1 else "bilinear"


def scale_image(img: np.ndarray, dw: int, dh: int, supersample: float, device: int = 0) -> np.ndarray:
    """The [H, W, 4] uint8 RGBA render scaled to [dh, dw, 4] as main.go:119-128
    does: into a fresh image with draw.Over, on the device."""
    f = scale_filter(supersample)
    if f is None:
        return img.copy()
    return _lib.scale_rgba(img, dw, dh, bilinear=f == "bilinear", device=device)


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
