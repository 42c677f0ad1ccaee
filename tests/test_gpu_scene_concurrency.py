"""One device scene rendered from several streams (and threads) at once.

Go's *Scene is read-only during Render (ray/tracer.go:48, ray/objects.go:37-46),
so several goroutines may render one scene concurrently. tray_scene_t gives the
same guarantee (include/tray.h, "Concurrency"): each render takes a launch
context of the scene (work queue, sample/chunk buffer, candidate records), and
a render that must reuse a busy context waits for it on the device. Every frame
below must equal, bit for bit, the same pass rendered alone and serially.
"""
import threading

import numpy as np
import pytest

from conftest import DEFAULT_BG, RICH_SETUP
from test_gpu_parity import bg_struct, camera

pytestmark = pytest.mark.gpu

# (camera setup, width, height, rays per pixel, first pass, passes, output)
SMALL = (RICH_SETUP, 48, 27, 64, 3, 2)
BIG = (np.array([0.5, 30, 0.25, 0, 0, 0, 0, 0, 1, 40.0, 10.0, 30.0, 0.0]), 160, 90, 64, 11, 4)
WIDE = (RICH_SETUP, 1280, 720, 64, 0, 1)  # ~5 ms: the renders enqueued after it overlap it


def _job(L, job, seed=2):
    setup, w, h, spp, first, n = job
    st = camera(L, setup, w, h)
    p = L.make_params(w, h, 50, spp, 0.5, seed, output=L.OUT_RGB_F32, pass_=first)
    return st, p, n, (n, h, w, 3)


def _serial(L, spheres, job):
    """Each pass rendered alone through the synchronous entry point."""
    st, p, n, shape = _job(L, job)
    frames = []
    for k in range(n):
        q = L.Params.from_buffer_copy(p)
        q.pass_ = p.pass_ + k
        frames.append(L.render(spheres, bg_struct(L, DEFAULT_BG), st, q, 0)[0])
    return np.stack(frames)


def _enqueue(L, torch, dev, job, stream):
    st, p, n, shape = _job(L, job)
    out = torch.full(shape, float("nan"), dtype=torch.float32, device="cuda")
    torch.cuda.current_stream().synchronize()  # the NaN fill has landed before another stream writes
    dev.render_passes_async(st, p, n, out.data_ptr(), stream.cuda_stream)
    return out


@pytest.mark.parametrize("contexts", [None, 1, 2])
def test_two_streams_one_scene(L, O, knobs, contexts):
    """Renders with different cameras, sizes and passes enqueued back to back on
    two streams on ONE scene. contexts = 1 serialises them through one launch
    context: the second render waits for the first on the device, then grows
    the context's chunk buffer (BIG needs more than SMALL) and rebuilds its
    candidate records for another camera; None (the default, 4) and 2 let them
    run concurrently in separate contexts."""
    import torch

    sc = O.rich_scene(2)
    if contexts is not None:
        knobs(scene_contexts=contexts)
    dev = L.DeviceScene(sc, bg_struct(L, DEFAULT_BG), 0)
    try:
        sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
        order = [(WIDE, sa), (SMALL, sb), (BIG, sa), (SMALL, sb), (BIG, sb), (SMALL, sa), (WIDE, sb), (BIG, sa)]
        st_s, p_s, n_s, _ = _job(L, SMALL)
        st_b, p_b, n_b, _ = _job(L, BIG)
        assert dev.plan(st_b, p_b, n_b).buffer_bytes > dev.plan(st_s, p_s, n_s).buffer_bytes  # a grow
        outs = [(job, _enqueue(L, torch, dev, job, stream)) for job, stream in order]
        torch.cuda.synchronize()
    finally:
        dev.release()
    want = {id(j): _serial(L, sc, j) for j in (SMALL, BIG, WIDE)}
    for i, (job, out) in enumerate(outs):
        got = out.cpu().numpy()
        assert np.array_equal(got, want[id(job)]), f"render {i} ({job[1]}x{job[2]}) differs from the serial render"


def test_context_grow_does_not_block_the_host(L, O, knobs):
    """A render that must grow a busy launch context's buffer only enqueues (VERDICT
    r5 item 5): with one context, a long render (8 C2 passes, ~40 ms) runs on stream
    A while tray_render_passes_async on stream B needs a bigger chunk buffer. B's
    call must return in < 2 ms of host time while A still runs (the old buffer is
    freed and the new one allocated in B's stream order, after A's render), and
    both frames must equal serial renders bit for bit."""
    import time

    import torch

    sc = O.rich_scene(2)
    knobs(scene_contexts=1)
    long_job = (RICH_SETUP, 1280, 720, 64, 0, 8)
    grow_job = (RICH_SETUP, 1280, 720, 64, 8, 12)
    dev = L.DeviceScene(sc, bg_struct(L, DEFAULT_BG), 0)
    try:
        sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
        st_l, p_l, n_l, shape_l = _job(L, long_job)
        st_g, p_g, n_g, shape_g = _job(L, grow_job)
        assert dev.plan(st_g, p_g, n_g).buffer_bytes > dev.plan(st_l, p_l, n_l).buffer_bytes
        # warm both streams and the pool (first use of a stream creates its hardware queue)
        _enqueue(L, torch, dev, SMALL, sa)
        _enqueue(L, torch, dev, SMALL, sb)
        torch.cuda.synchronize()
        out_l = torch.full(shape_l, float("nan"), dtype=torch.float32, device="cuda")
        out_g = torch.full(shape_g, float("nan"), dtype=torch.float32, device="cuda")
        torch.cuda.synchronize()
        dev.render_passes_async(st_l, p_l, n_l, out_l.data_ptr(), sa.cuda_stream)
        a_done = torch.cuda.Event()
        a_done.record(sa)
        t0 = time.perf_counter()
        dev.render_passes_async(st_g, p_g, n_g, out_g.data_ptr(), sb.cuda_stream)
        host_ms = (time.perf_counter() - t0) * 1e3
        a_running = not a_done.query()
        torch.cuda.synchronize()
    finally:
        dev.release()
    assert a_running, "the long render ended before the grow was enqueued: nothing was measured"
    assert host_ms < 2.0, f"tray_render_passes_async with a context grow took {host_ms:.3f} ms of host time"
    assert np.array_equal(out_l.cpu().numpy(), _serial(L, sc, long_job))
    assert np.array_equal(out_g.cpu().numpy(), _serial(L, sc, grow_job))


def test_threads_enqueue_on_one_scene(L, O):
    """Four threads each enqueue renders of one scene on a stream of their own
    (ctypes releases the GIL around every call): more renders in flight than
    the scene's four contexts, so some wait for a context on the device."""
    import torch

    sc = O.rich_scene(2)
    dev = L.DeviceScene(sc, bg_struct(L, DEFAULT_BG), 0)
    jobs = [SMALL, BIG, SMALL, BIG]
    results = [[] for _ in jobs]
    errors = []

    def work(t):
        try:
            s = torch.cuda.Stream()
            with torch.cuda.stream(s):
                for _ in range(3):
                    results[t].append(_enqueue(L, torch, dev, jobs[t], s))
        except BaseException as e:  # noqa: BLE001 - reported below
            errors.append(e)

    try:
        threads = [threading.Thread(target=work, args=(t,)) for t in range(len(jobs))]
        for th in threads:
            th.start()
        for th in threads:
            th.join()
        torch.cuda.synchronize()
    finally:
        dev.release()
    assert not errors, errors
    want = {id(j): _serial(L, sc, j) for j in (SMALL, BIG)}
    for t, job in enumerate(jobs):
        for out in results[t]:
            assert np.array_equal(out.cpu().numpy(), want[id(job)])


def test_release_waits_for_enqueued_renders(L, O):
    """tray_scene_release with renders still enqueued on two streams waits for
    them (their contexts' events) before freeing the buffers they use."""
    import torch

    sc = O.rich_scene(2)
    dev = L.DeviceScene(sc, bg_struct(L, DEFAULT_BG), 0)
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    a = _enqueue(L, torch, dev, WIDE, sa)
    b = _enqueue(L, torch, dev, BIG, sb)
    dev.release()  # must not free what the two renders still use
    torch.cuda.synchronize()
    assert np.array_equal(a.cpu().numpy(), _serial(L, sc, WIDE))
    assert np.array_equal(b.cpu().numpy(), _serial(L, sc, BIG))
