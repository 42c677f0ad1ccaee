"""The kernel's division by launch-invariant integers (FastDiv in
tray_amd/csrc/tray_kernel.hpp: work-item decoding by frame_items, rays per
pixel and tiles per row; compact row -> image row by tile_rows), restated here
with Python integers: make_fastdiv on the host and udiv on the device must give
n // d and n % d for every 32-bit n. Frames decoded this way are checked bit for
bit against the oracle by the GPU parity tests."""
import re

import numpy as np

from conftest import ROOT

M32 = (1 << 32) - 1


def make_fastdiv(d):  # tray_kernel.hpp make_fastdiv
    l = 0
    while l < 32 and (1 << l) < d:
        l += 1
    m = ((1 << 32) * ((1 << l) - d)) // d + 1
    return d, m & M32, min(l, 1), max(l - 1, 0)


def udiv(n, f):  # tray_kernel.hip udiv (32-bit unsigned arithmetic)
    d, m, s1, s2 = f
    t = (n * m) >> 32
    q = ((t + (((n - t) & M32) >> s1)) & M32) >> s2
    return q, (n - q * d) & M32


def test_header_restatement_matches():
    src = open(f"{ROOT}/tray_amd/csrc/tray_kernel.hpp").read()
    assert "(1ull << 32) * ((1ull << l) - d)) / d + 1" in src
    assert re.search(r"f\.s1 = l < 1 \? l : 1;\s*f\.s2 = l > 1 \? l - 1 : 0;", src)


def test_fastdiv_exact():
    rng = np.random.default_rng(3)
    divisors = list(range(1, 2049)) + [2 ** k + e for k in range(1, 32) for e in (-1, 0, 1)] + \
        [M32, 2 ** 31 + 1, 3 * 2 ** 30] + [int(v) for v in rng.integers(1, 2 ** 32, 2000, dtype=np.uint64)]
    for d in divisors:
        d = int(min(max(d, 1), M32))
        f = make_fastdiv(d)
        ns = [0, 1, d - 1, d, d + 1, 2 * d - 1, 2 * d, M32, M32 - 1, M32 - d % (M32 + 1)] + \
            [int(v) for v in rng.integers(0, 2 ** 32, 64, dtype=np.uint64)]
        for n in ns:
            n = n & M32
            assert udiv(n, f) == (n // d, n % d), (n, d)
