import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) device; runs the HIP path through the C-ABI")


def _ensure_built():
    # Built artefacts travel to the GPU box with the snapshot; build here if absent.
    if not os.path.exists(os.path.join(ROOT, "oracle", "libtray_oracle.so")):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    if not os.path.exists(os.path.join(ROOT, "tray_amd", "libtray_amd.so")):
        subprocess.run(["make", "-s", "-j4", "-C", os.path.join(ROOT, "tray_amd")], check=True)


_ensure_built()

# torch ships its own HIP runtime. If libtray_amd.so (linked against /opt/rocm's)
# initialises HIP first in a process, torch then finds no GPU; loading torch
# first makes both share torch's runtime. GPU tests use torch for device buffers.
try:
    import torch  # noqa: F401
except ImportError:  # the CPU suite does not need it
    pass


@pytest.fixture(scope="session")
def O():
    from oracle import oracle

    return oracle


@pytest.fixture(scope="session")
def L():
    from tray_amd import _lib

    return _lib


@pytest.fixture
def knobs(L):
    """include/tray_debug.h knobs for one test (`knobs(acc_slots=0)`), all cleared afterwards."""
    yield lambda **kw: L.set_debug_knobs(**kw)
    L.clear_debug_knobs()


def load_golden(name):
    return dict(np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False))


def example_sky_mask():
    """tests/golden/example_sky_mask.npz: the pixels of example.png no camera ray of
    any RichScene can reach a sphere from (tests/golden/make_sky_mask.py), their
    bytes in row-major order, and the rows to render to cover them."""
    g = load_golden("example_sky_mask")
    h, w = (int(v) for v in g["shape"])
    mask = np.unpackbits(g["mask"])[: h * w].reshape(h, w).astype(bool)
    return mask, g["rgb"], int(np.nonzero(mask.any(1))[0].max()) + 1


RICH_SETUP = np.array([13, 2, 3, 0, 0, 0, 0, 1, 0, 20.0, 10.0, 10.0, 0.1])  # RichSceneCamera, camera.go:144-154
DEFAULT_BG = np.array([1.0, 1.0, 1.0, 0.4, 0.65, 1.0])  # DefaultBackground, objects.go:106-110


def srgb_boundary_distance(linear):
    """|frac(255 * s) - 0.5| per channel, s = the sRGB transfer of a linear colour
    (ray/vec3.go:173-180 via fortio.org/terminal LinearToSrgb, IEC form): how far
    the 8-bit encoder's rounding is from flipping. A +-1 LSB difference against
    the reference's own example.png can only come from noise where this is small."""
    c = np.clip(np.asarray(linear, dtype=np.float64), 0.0, 1.0)
    s = 255.0 * np.where(c <= 0.0031308, 12.92 * c, 1.055 * np.power(c, 1 / 2.4) - 0.055)
    return np.abs(s - np.floor(s) - 0.5)


# example.png pins (tests/golden/example_sky_rows.npz, rows 0..48 = pure sky):
#  * pixel-centre pinhole rays (no random stream involved in the sky colour)
#    must give the reference's bytes EXACTLY, except channels whose encoded
#    value lies within SKY_EDGE_PINHOLE of a rounding boundary (arm64 Go fuses
#    multiply-adds in the camera: ulp-level differences; measured misses all lie
#    within 0.0343 of a boundary);
#  * the r=64 render (anti-aliasing on a different random stream than
#    fortio.org/rand) may differ by 1 LSB only within SKY_EDGE_AA of a boundary
#    (measured misses: 915 channels, all within 0.0547).
SKY_EDGE_PINHOLE = 0.04
SKY_EDGE_AA = 0.06
