"""The arithmetic argument behind the kernel's fixed-point pixel sums (DESIGN.md
§5 "Accumulation"; tray_kernel.hip end_path / acc_retire / resolve_kernel),
checked on the CPU with numpy FP64: a sample colour c, |c| < 2^e, scaled by 2^k
(k = 47 - e) and rounded to an integer v = rint(c 2^k) has |v| <= 2^47, so any
sum of <= 64 of them is an exact FP64 integer: the same bits in every order and
for every split into sub-accumulators; the pixel total over several 64-sample
chunks is an exact int64 sum; the mean is within 2^-(k+1) of the exact mean
(one more rounding for the conversion and the 1/r product); a NaN propagates."""
import math

import numpy as np
import pytest

K_BITS = 47


def chunk_sum(v, order, copies=1):
    """FP64 adds in `order` into `copies` accumulators (lane % copies), then their sum."""
    acc = [0.0] * copies
    for lane, i in enumerate(order):
        acc[lane % copies] += float(v[i])
    total = 0.0
    for a in acc:
        total += a
    return total


@pytest.mark.parametrize("e", [0, 1, 3])
def test_chunk_sums_are_exact_in_any_order(e):
    rng = np.random.default_rng(7 + e)
    k = K_BITS - e
    for _ in range(20):
        c = rng.uniform(-1, 1, 64) * (2.0 ** e) * 0.999
        v = np.rint(np.ldexp(c, k))
        assert np.max(np.abs(v)) <= 2.0 ** K_BITS
        exact = math.fsum(v)
        sums = {chunk_sum(v, rng.permutation(64), copies) for copies in (1, 2, 4) for _ in range(8)}
        assert sums == {exact}
        # beyond the bound (one extra bit) the order starts to matter: the bound is needed
        w = np.rint(np.ldexp(c, k + 8))
        assert len({chunk_sum(w, rng.permutation(64)) for _ in range(64)}) > 1


def test_pixel_total_and_mean_error():
    rng = np.random.default_rng(11)
    e, r = 1, 256
    k = K_BITS - e
    for _ in range(10):
        c = rng.uniform(0, 1.0, r)  # colours of one pixel's r samples, bound 1.001 < 2^1
        v = np.rint(np.ldexp(c, k))
        chunks = [chunk_sum(v[i:i + 64], rng.permutation(64), 2) for i in range(0, r, 64)]
        total = sum(int(x) for x in chunks)  # the resolve pass: int64 adds of exact chunk sums
        assert total == sum(int(x) for x in v)  # exact (the total may exceed 2^53: no FP64 rounding)
        mean = math.ldexp(float(total), -k) * (1.0 / r)
        exact_mean = math.fsum(c) / r
        assert abs(mean - exact_mean) <= 2.0 ** -(k + 1) + 4 * 2.0 ** -53 * abs(exact_mean)
        # Go's sequential FP64 sum (ray/tracer.go:143) differs from the exact mean by its own roundings
        seq = 0.0
        for x in c:
            seq += float(x)
        assert abs(seq * (1.0 / r) - exact_mean) <= r * 2.0 ** -53


def test_nan_sample_poisons_its_channel():
    v = np.rint(np.ldexp(np.linspace(0, 0.5, 64), 46))
    v[17] = np.nan
    assert math.isnan(chunk_sum(v, range(64), 2))
