"""The exact path bench.py times, checked against the oracle at its own size.

bench.py (`launch`/`frames`) renders F = 16 progressive passes per launch
through tray_render_passes_async into TRAY_OUT_RGB_F32, with two frame slots
(own output and stream, ONE DeviceScene whose launch context per stream holds
the work queue and chunk records) in flight at once, and with 64 | r every pixel's samples summed on chip
as exact fixed-point chunk sums ("Accumulation"). This test runs
that shape for C2 (the headline) and C5 (dense scene: LDS layout 2, four
64-sample chunks per pixel):

  launch A: slot 0, passes  0..15     (in flight together with B)
  launch B: slot 1, passes 16..31
  launch C: slot 0, passes 32..47     (slot 0's context again: its work queue
                                       must have been re-zeroed by A's resolve)

and checks frames 0, 7, 15 of A, 0 and 15 of B and 15 of C (passes 0, 7, 15,
16, 31, 47):
  * each whole frame equals, bit for bit, a single-pass tray_render_async of
    pass k into RGB_F32 (what the other parity tests check),
  * that render's per-pixel Scene.Hit counts equal the oracle's at >= 256
    picked pixels (random, longest paths, ground rows, band edges),
  * the bench frame's colours at those pixels equal float32 of the oracle's
    FP64 mean (ray/tracer.go:120-155 restated, pass k) within one f32 rounding
    of a value inside 1e-12 of it (north-star gate 1e-4).
"""
import numpy as np
import pytest

from test_gpu_configs import WORKERS, picks  # noqa: F401  (shared pixel picks)

pytestmark = pytest.mark.gpu

F = 16
CHECKS = {  # launch -> (first pass, slot, frames checked)
    "A": (0, 0, (0, 7, 15)),
    "B": (16, 1, (0, 15)),
    "C": (32, 0, (15,)),
}


def _oracle(O, spheres, cam, W, H, spp, depth, seed, xs, ys, pass_):
    from concurrent.futures import ThreadPoolExecutor

    from conftest import DEFAULT_BG

    parts = np.array_split(np.arange(len(xs)), WORKERS)
    with ThreadPoolExecutor(WORKERS) as ex:
        res = list(ex.map(lambda ix: O.render_pixels(spheres, DEFAULT_BG, cam._state.as_array(), W, H, spp, depth,
                                                     0.5, seed, xs[ix], ys[ix], pass_=pass_), parts))
    return np.concatenate([r[0] for r in res]), np.concatenate([r[1] for r in res])


@pytest.mark.parametrize("config", ["c2", "c5"])
def test_bench_launch_shape_vs_oracle(L, O, config):
    import torch

    from bench import CONFIGS
    from tray_amd import ray

    _, seed, half, W, H, spp, depth = CONFIGS[config]
    spheres = ray.rich_scene_array(seed, half)
    cam = ray.RichSceneCamera()
    cam.Initialize(W, H)
    bg = ray._background(ray.DefaultBackground())
    params = L.make_params(W, H, depth, spp, 0.5, seed, output=L.OUT_RGB_F32)
    scene = L.DeviceScene(spheres, bg, 0)  # one scene, two streams (bench.py)
    try:
        plan = scene.plan(cam._state, params, F).as_dict()
        assert plan["acc_slots"] > 0 and plan["fixed_point_shift"] > 0, plan  # the on-chip sums bench.py times
        if config == "c5":
            assert plan["lds_layout"] == 2, plan
        streams = [torch.cuda.current_stream(), torch.cuda.Stream()]
        outs = {k: torch.empty((F, H, W, 3), dtype=torch.float32, device="cuda") for k in CHECKS}
        for name, (first, slot, _) in CHECKS.items():  # enqueued back to back: A and B overlap, C follows A
            p = L.Params.from_buffer_copy(params)
            p.pass_ = first
            with torch.cuda.stream(streams[slot]):
                scene.render_passes_async(cam._state, p, F, outs[name].data_ptr(), streams[slot].cuda_stream)
        torch.cuda.synchronize()
        rng = np.random.default_rng({"c2": 42, "c5": 57}[config])
        single = torch.empty((H, W, 3), dtype=torch.float32, device="cuda")
        seg = torch.empty((H, W), dtype=torch.int32, device="cuda")
        stream = torch.cuda.current_stream().cuda_stream
        for name, (first, slot, frames) in CHECKS.items():
            for f in frames:
                k = first + f
                bench_frame = outs[name][f]
                p = L.Params.from_buffer_copy(params)
                p.pass_ = k
                scene.render_async(cam._state, p, single.data_ptr(), seg.data_ptr(), stream)
                torch.cuda.synchronize()
                assert torch.equal(bench_frame, single), f"{config} pass {k}: passes launch != single render"
                got = bench_frame.cpu().numpy()
                assert np.isfinite(got).all()
                seg_host = seg.cpu().numpy().astype(np.uint32)
                assert seg_host.min() >= spp and seg_host.max() <= spp * depth
                xs, ys = picks(seg_host, W, H, spp, rng)
                assert len(xs) >= 256
                ref, rseg = _oracle(O, spheres, cam, W, H, spp, depth, seed, xs, ys, k)
                assert np.array_equal(seg_host[ys, xs], rseg), \
                    f"{config} pass {k}: {int((seg_host[ys, xs] != rseg).sum())} pixels took different paths"
                g = got[ys, xs].astype(np.float64)
                assert float(np.abs(g - ref).max()) <= 1e-4  # north-star gate
                # f32 output: one rounding of a value within 1e-12 of the oracle's mean
                tol = np.abs(ref) * 2.0**-24 + 1e-12
                assert np.all(np.abs(g - ref) <= tol), f"{config} pass {k}: {float(np.abs(g - ref).max())}"
                assert (got[ys, xs] == ref.astype(np.float32)).mean() >= 0.999
    finally:
        scene.release()
