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


def load_golden(name):
    return dict(np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False))


RICH_SETUP = np.array([13, 2, 3, 0, 0, 0, 0, 1, 0, 20.0, 10.0, 10.0, 0.1])  # RichSceneCamera, camera.go:144-154
DEFAULT_BG = np.array([1.0, 1.0, 1.0, 0.4, 0.65, 1.0])  # DefaultBackground, objects.go:106-110
