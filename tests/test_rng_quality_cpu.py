"""The renderer's draw RNG (include/tray.h "Counter RNG contract", ABI 6): a keyed
pcg4d block (Jarzynski & Olano, "Hash Functions for GPU Rendering", JCGT 9(3),
2020) with an xorshift-16 of each output word. The C oracle's draw_key/draw_block
against an independent numpy restatement written from the contract text, and the
statistical checks the change from Philox4x32-10 was made under (a Philox block
was ~7.6 % of the C2 frame): per-bit bias, strict avalanche over every counter
bit the renderer varies (pixel, sample, bounce, purpose), correlation between
the words of a block and between neighbouring counters. The reference's own
sampler statistics (ray/vec3_test.go:539-741) run on the new draws in
tests/test_oracle_sampler_golden.py. CPU only."""
import numpy as np
import pytest

M = np.uint32


def ph_key(seed):  # Philox4x32-10 of (0, 0, 0, 5 << 24) keyed by the seed (the draw key)
    c = [M(0), M(0), M(0), M(5 << 24)]
    k0, k1 = M(seed & 0xFFFFFFFF), M(seed >> 32)
    for r in range(10):
        if r:
            k0, k1 = M((int(k0) + 0x9E3779B9) & 0xFFFFFFFF), M((int(k1) + 0xBB67AE85) & 0xFFFFFFFF)
        p0, p1 = 0xD2511F53 * int(c[0]), 0xCD9E8D57 * int(c[2])
        c = [M((p1 >> 32) ^ int(c[1]) ^ int(k0)), M(p1 & 0xFFFFFFFF), M((p0 >> 32) ^ int(c[3]) ^ int(k1)),
             M(p0 & 0xFFFFFFFF)]
    return tuple(int(v) for v in c)


def block(key, pixel, sample, bounce, purpose):
    """numpy restatement of the contract's draw block (vectorised over the counters)."""
    with np.errstate(over="ignore"):
        v = [np.asarray(x, dtype=M) ^ M(k) for x, k in zip((pixel, sample, bounce, purpose), key)]
        v = [x * M(1664525) + M(1013904223) for x in v]
        for _ in range(2):
            v[0] = v[0] + v[1] * v[3]
            v[1] = v[1] + v[2] * v[0]
            v[2] = v[2] + v[0] * v[1]
            v[3] = v[3] + v[1] * v[2]
            v = [x ^ (x >> M(16)) for x in v]
    return np.stack(v)


@pytest.mark.parametrize("seed", [0, 2, 7, 0xFFFFFFFF, 1 << 40, (1 << 64) - 1])
def test_oracle_draws_equal_restatement(O, seed):
    key = O.draw_key(seed)
    assert key == ph_key(seed)
    rng = np.random.default_rng(seed % 1000 + 1)
    for _ in range(200):
        c = (int(rng.integers(0, 2**32)), int(rng.integers(0, 2**32)), int(rng.integers(0, 64)),
             int(rng.choice([1, 3])))
        assert O.draw_block(key, *c) == tuple(int(x) for x in block(key, *c))


def _counters(n, rng):
    return [rng.integers(0, 1 << 24, n).astype(M), rng.integers(0, 1 << 24, n).astype(M),
            rng.integers(0, 64, n).astype(M), rng.choice(np.array([1, 3], dtype=M), n)]


def test_bit_bias_and_word_correlation():
    n = 1 << 20
    rng = np.random.default_rng(3)
    out = block(ph_key(2), *_counters(n, rng))
    bits = ((out[:, :, None] >> np.arange(32, dtype=M)) & M(1)).mean(1)
    assert np.abs((bits - 0.5) / np.sqrt(0.25 / n)).max() < 5.5  # 128 bits, none biased beyond noise
    u = out.astype(np.float64) * 2.0**-32
    corr = np.corrcoef(u)[np.triu_indices(4, 1)]
    assert np.abs(corr).max() < 5.0 / np.sqrt(n)


def test_neighbouring_counters_uncorrelated():
    """Adjacent pixels, samples and bounces (what a wave draws side by side)."""
    n = 1 << 20
    rng = np.random.default_rng(4)
    key = ph_key(2)
    c = _counters(n, rng)
    a = block(key, *c).astype(np.float64) * 2.0**-32
    for word in range(3):
        d = [x.copy() for x in c]
        d[word] = d[word] + M(1)
        b = block(key, *d).astype(np.float64) * 2.0**-32
        for w in range(4):
            assert abs(np.corrcoef(a[w], b[w])[0, 1]) < 5.0 / np.sqrt(n), (word, w)


def test_strict_avalanche_on_the_varied_counter_bits():
    """Flipping any counter bit the renderer varies (pixel and sample bits 0-23,
    bounce 0-5, purpose 1 <-> 3) flips every output bit with probability 1/2
    within noise. Without the final xorshift, pcg4d's low output bits fail this
    (a flip of counter bit 17 never reaches output bit 0)."""
    n = 1 << 16
    rng = np.random.default_rng(5)
    keys = np.stack([np.array(ph_key(int(s)), dtype=M) for s in rng.integers(0, 2**63, 8)])
    worst = 0.0
    for word, nbits in ((0, 24), (1, 24), (2, 6), (3, 1)):
        for bit in range(nbits):
            key = keys[bit % len(keys)]
            c = _counters(n, rng)
            base = block(key, *c)
            d = [x.copy() for x in c]
            d[word] = d[word] ^ M(2 if word == 3 else 1 << bit)
            flips = block(key, *d) ^ base
            p = ((flips[:, :, None] >> np.arange(32, dtype=M)) & M(1)).mean(1)
            worst = max(worst, float(np.abs(p - 0.5).max()))
    assert worst < 5.0 * 0.5 / np.sqrt(n), worst
