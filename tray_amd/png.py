"""PNG sink for rendered frames: the host side of `png.Encode(f, img)` in the
reference's CLIs (benchmark/benchmark.go:23-33, main.go:26-36), which encode the
*image.RGBA that Tracer.Render returns. Standard library only (zlib): 8-bit RGBA,
non-interlaced, filter type 0 on every row."""
from __future__ import annotations

import struct
import zlib

import numpy as np


def _chunk(kind: bytes, data: bytes) -> bytes:
    return struct.pack(">I", len(data)) + kind + data + struct.pack(">I", zlib.crc32(kind + data) & 0xFFFFFFFF)


def encode_png(rgba: np.ndarray, level: int = 6) -> bytes:
    """PNG bytes of an [H, W, 4] uint8 image (Tracer.imageData / TRAY_OUT_RGBA8 rows)."""
    img = np.ascontiguousarray(rgba)
    if img.dtype != np.uint8 or img.ndim != 3 or img.shape[2] != 4:
        raise ValueError("expected an [H, W, 4] uint8 RGBA image")
    h, w = img.shape[:2]
    raw = np.zeros((h, 1 + 4 * w), dtype=np.uint8)  # filter byte 0 + row
    raw[:, 1:] = img.reshape(h, 4 * w)
    ihdr = struct.pack(">IIBBBBB", w, h, 8, 6, 0, 0, 0)  # 8-bit, colour type 6 (RGBA)
    return (b"\x89PNG\r\n\x1a\n" + _chunk(b"IHDR", ihdr) + _chunk(b"IDAT", zlib.compress(raw.tobytes(), level))
            + _chunk(b"IEND", b""))


def save_png(path: str, rgba: np.ndarray) -> None:
    with open(path, "wb") as f:
        f.write(encode_png(rgba))


def decode_png(data: bytes) -> np.ndarray:
    """Inverse of encode_png for 8-bit RGBA, filter-0 images (tests)."""
    if data[:8] != b"\x89PNG\r\n\x1a\n":
        raise ValueError("not a PNG")
    pos, w, h, idat = 8, 0, 0, b""
    while pos < len(data):
        (n,) = struct.unpack(">I", data[pos:pos + 4])
        kind, body = data[pos + 4:pos + 8], data[pos + 8:pos + 8 + n]
        if zlib.crc32(kind + body) & 0xFFFFFFFF != struct.unpack(">I", data[pos + 8 + n:pos + 12 + n])[0]:
            raise ValueError("bad CRC")
        if kind == b"IHDR":
            w, h, depth, ctype = struct.unpack(">IIBB", body[:10])
            if (depth, ctype) != (8, 6):
                raise ValueError("only 8-bit RGBA")
        elif kind == b"IDAT":
            idat += body
        pos += 12 + n
    raw = np.frombuffer(zlib.decompress(idat), dtype=np.uint8).reshape(h, 1 + 4 * w)
    if np.any(raw[:, 0] != 0):
        raise ValueError("only filter type 0")
    return raw[:, 1:].reshape(h, w, 4).copy()
