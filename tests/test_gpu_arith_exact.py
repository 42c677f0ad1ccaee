"""The kernel's shortcuts for correctly rounded arithmetic are bit-identical to
the full forms, checked on the device (the tools/ checkers, built by
__graft_entry__.build()):

- sqrt_cr / rcp_cr (tray_amd/csrc/fp64.hpp) == the compiler's sqrt and 1.0/x
  over 4.3e9 random and edge-case operands (tools/sqrt_rcp_check.hip);
- sincos_2pi_word(w) == sincos_2pi(w 2^-32) for all 2^32 words
  (tools/sincos_check.hip), the sampler contract of include/tray.h;
- Markstein's division by a correctly rounded reciprocal == a / b
  (tools/div_check.hip; the kernel's div_rcp).

Together with the oracle parity tests these pin the kernel's FP64 results to
the reference arithmetic without tolerance."""
import json
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu

TOOLS = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools")


def run_checker(name):
    exe = os.path.join(TOOLS, name)
    if not os.path.exists(exe):
        pytest.skip(f"tools/{name} not built (make -C tools)")
    out = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    lines = [json.loads(l) for l in out.stdout.splitlines() if l.startswith("{")]
    assert lines, out.stdout + out.stderr
    return lines


def test_sqrt_rcp_shortcuts_are_exact():
    rows = run_checker("sqrt_rcp_check")
    assert sum(r["operands"] for r in rows) > 4_000_000_000
    assert all(r["sqrt_mismatches"] == 0 and r["rcp_mismatches"] == 0 for r in rows), rows


def test_sincos_word_form_is_exact_for_every_word():
    (row,) = run_checker("sincos_check")
    assert row["words"] == 2**32 and row["mismatches"] == 0, row


def test_markstein_division_is_exact():
    rows = run_checker("div_check")
    assert all(r["mismatches"] == 0 for r in rows), rows
