"""Terminal sink (tray_amd/terminal.py, main.go:86-131): host-side properties
only — parity unpinned (x/image/draw and fortio.org/terminal are absent and the
reference holds no fixture for them)."""
import numpy as np

from tray_amd import terminal


def rgba(h, w, seed=0):
    rng = np.random.default_rng(seed)
    img = rng.integers(0, 256, (h, w, 4), dtype=np.uint8)
    img[..., 3] = 255
    return img


def test_image_size_follows_main_go():
    assert terminal.image_size(80, 24, 4) == (320, 192)   # main.go:88, two pixel rows per text row
    assert terminal.image_size(80, 24, 0) == (80, 48)     # -s <= 0 means 1 (main.go:63-66)
    assert terminal.image_size(3, 1, 0.5) == (2, 1)       # Go math.Round: halves away from zero


def test_scale_identity_and_constant():
    img = rgba(6, 10)
    assert np.array_equal(terminal.scale_image(img, 10, 6), img)
    flat = np.full((40, 64, 4), (200, 17, 90, 255), dtype=np.uint8)
    assert np.array_equal(terminal.scale_image(flat, 16, 10), flat[:10, :16])  # weights sum to 1


def test_scale_down_is_box_like_average():
    # 2x shrink of a checkerboard: every output pixel sees as much black as white
    img = np.zeros((8, 8, 4), dtype=np.uint8)
    img[..., 3] = 255
    img[(np.indices((8, 8)).sum(0) % 2) == 0, :3] = 255
    out = terminal.scale_image(img, 4, 4)
    assert np.all(np.abs(out[..., :3].astype(int) - 127) <= 24) and np.all(out[..., 3] == 255)


def test_scale_up_is_nearest():
    img = rgba(3, 4)
    out = terminal.scale_image(img, 8, 6)  # supersample < 1 (main.go:122)
    assert np.array_equal(out, np.repeat(np.repeat(img, 2, 0), 2, 1))


def test_weights_rows_normalised():
    for dw, sw in [(7, 31), (16, 64), (5, 5), (1, 9)]:
        w = terminal._weights(dw, sw, False)
        assert np.allclose(w.sum(1), 1.0) and np.all(w >= 0)


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
