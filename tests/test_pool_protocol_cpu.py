"""The work queue's reservation protocol (tray_kernel.hip take_chunk and the
refill loop), restated step for step and run under random interleavings of the
waves of one workgroup: every chunk of the launch is handed out exactly once,
no chunk past the end is, and every wave stops (its take sees kPoolDone).

Device protocol (one 64-bit LDS word per workgroup: end << 32 | next):
  * a take adds G to `next` atomically and reads (next, end) from the result;
  * next + G <= end: the wave owns [next, next + G);
  * next <= end < next + G (exactly one take per pool covers its end): the wave
    refills the pool from the global queue (atomicAdd of pool_chunks) and owns
    [next, end) when next < end;
  * next > end: the wave sleeps until `end` changes, then takes again;
  * a refill past the launch's chunks stores end = kPoolDone; every later take
    returns kPoolDone.
G is the wave's reservation size: wave_chunks while its last reservation ended
before late_at, 1 afterwards (launch_render sets both)."""
import random

import pytest

DONE = 0xFFFFFFFF


class Pool:
    def __init__(self, nchunks, pool_chunks):
        self.nchunks, self.pool_chunks = nchunks, pool_chunks
        self.word_next, self.word_end = 0, 0  # an empty pool: the first taker refills
        self.queue = 0

    def refill(self):
        base = self.queue
        self.queue += self.pool_chunks
        if base >= self.nchunks:
            self.word_next, self.word_end = 0, DONE
        else:
            self.word_next, self.word_end = base, min(base + self.pool_chunks, self.nchunks)


def wave(pool, G_of, got):
    """One wave's takes as a generator: yields between atomic steps."""
    grp_end = 0
    while True:
        G = G_of(grp_end)
        nxt, end = pool.word_next, pool.word_end  # fetch_add returns the old word
        pool.word_next = (pool.word_next + G) & 0xFFFFFFFF
        yield
        if end == DONE:
            return
        if nxt + G <= end:
            got.extend(range(nxt, nxt + G))
            grp_end = nxt + G
            yield
            continue
        if nxt <= end:
            pool.refill()
            yield
            if nxt < end:
                got.extend(range(nxt, end))
                grp_end = end
                yield
            continue
        while pool.word_end == end:  # sleep until the refill changes `end`
            yield


@pytest.mark.parametrize("nchunks,pool_chunks,G,waves,late_at", [
    (1000, 64, 32, 16, 600), (1000, 64, 32, 16, 0), (1000, 64, 1, 16, 0), (999, 64, 32, 5, 900),
    (37, 16, 8, 16, 10), (5, 16, 32, 16, 0), (4096, 64, 3, 7, 4000), (64, 64, 64, 2, 64), (1, 16, 32, 3, 0)])
def test_every_chunk_exactly_once(nchunks, pool_chunks, G, waves, late_at):
    for seed in range(40):
        rng = random.Random(seed)
        pool = Pool(nchunks, pool_chunks)
        got = []
        G_of = (lambda grp_end: 1 if grp_end >= late_at else G)
        gens = [wave(pool, G_of, got) for _ in range(waves)]
        live = list(gens)
        steps = 0
        while live:
            g = rng.choice(live)
            try:
                next(g)
            except StopIteration:
                live.remove(g)
            steps += 1
            assert steps < 10_000_000, "a wave never stopped"
        assert sorted(got) == list(range(nchunks)), (seed, len(got))
