"""include/tray.h from C: a C99 program (tests/c/tray_c_caller.c) compiled with
gcc -std=c99 -Wall -Wextra -Werror -pedantic against the header and linked with
libtray_amd.so, the way a cgo shim binds it. Proves the header
is C (no C++ constructs), the entry points link from C, host setup works from C,
and a C progress callback is driven by tray_render_progress."""
import os
import subprocess

import pytest

from conftest import ROOT


def _run_caller(tmp_path):
    exe = str(tmp_path / "tray_c_caller")
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Wextra", "-Werror", "-pedantic", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "c", "tray_c_caller.c"), "-L", os.path.join(ROOT, "tray_amd"),
                    "-ltray_amd", "-Wl,-rpath," + os.path.join(ROOT, "tray_amd"), "-o", exe], check=True)
    res = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert res.returncode == 0, res.stdout + res.stderr
    out = {}
    for line in res.stdout.splitlines():
        for kv in line.split():
            k, _, v = kv.partition("=")
            out[k] = v
    return out


def _check_host_side(out):
    assert out["abi"] == "6" and out["spheres"] == "486" and out["rows"] == "9"
    assert out["focus"] == "10"
    assert out["srgb"] == "0,188,255,10,0,255"  # ray/vec3_test.go:264-289: 0, 0.5 -> 188, 1, clamps
    assert out["bad_width"] == "-1" and out["bad_reserved"] == "-1"  # TRAY_ERR_INVALID_ARGUMENT


@pytest.mark.skipif(os.path.exists("/dev/kfd"), reason="a GPU is present (see the gpu variant)")
def test_c99_caller_without_device(tmp_path):
    out = _run_caller(tmp_path)
    _check_host_side(out)
    assert out["devices"] == "0"
    assert out["render"] == "-4" and out["render_progress"] == "-4"  # TRAY_ERR_NO_DEVICE: no fallback
    assert out["progress_rows"] == "0"


@pytest.mark.gpu
def test_c99_caller_on_device(tmp_path):
    out = _run_caller(tmp_path)
    _check_host_side(out)
    assert int(out["devices"]) >= 1
    assert out["render"] == "0" and out["render_progress"] == "0"
    assert out["progress_rows"] == "9"  # every row reported exactly once
