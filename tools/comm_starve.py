#!/usr/bin/env python3
"""Does a collective that follows each launch starve behind the next persistent
render grid? (round 5; one GPU, numbers are a rehearsal)

bench.py --gpus N renders rank k's row tiles 16 frames per launch on two frame
slots and, after each launch, gathers its frames to rank 0 with RCCL on a stream
of its own; the next launch into the same slot waits for that gather. RCCL's
gather runs as kernels, and a render grid that holds every CU (one 1024-lane
workgroup per CU, the VGPR file full) leaves them no room until it drains. This
tool replays one rank's side of that pipeline on one GPU with a stand-in for the
gather: an elementwise kernel over `--comm-mb` MB on the comm stream after every
launch (rank 0 of an 8-way C2 split receives ~155 MB per 16-frame launch, the
others send ~22 MB). It reports ms per frame for

  render only        no comm kernel (tools/shard_sim.py's number)
  comm               the stand-in after every launch, slot reuse waits for it
  comm + reserve K   the same with the render grid leaving K workgroup slots
                     free ("grid_reserve" knob), so the comm kernel runs beside it

    python tools/comm_starve.py [--n 8] [--comm-mb 155] [--reserve 0,1,8] [--launches 12]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--n", type=int, default=8, help="ranks of the split (rank 0's rows are rendered)")
    ap.add_argument("--passes", type=int, default=16)
    ap.add_argument("--launches", type=int, default=12)
    ap.add_argument("--comm-mb", type=float, default=155.0)
    ap.add_argument("--reserve", default="0,1,8")
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    import numpy as np
    import torch

    from bench import CONFIGS
    from tray_amd import _lib, ray, shard

    _, seed, half, W, H, spp, depth = CONFIGS[args.config]
    spheres = ray.rich_scene_array(seed, half)
    cam = ray.RichSceneCamera()
    cam.Initialize(W, H)
    scene = _lib.DeviceScene(spheres, ray._background(ray.DefaultBackground()), 0)
    params = shard.shard_params(_lib.make_params(W, H, depth, spp, 0.5, seed, output=_lib.OUT_RGB_F32), 1,
                                args.n, 0) if args.n > 1 else _lib.make_params(W, H, depth, spp, 0.5, seed,
                                                                              output=_lib.OUT_RGB_F32)
    rows = _lib.params_rows(params)
    F = args.passes
    outs = [torch.empty((F, rows, W, 3), dtype=torch.float32, device="cuda") for _ in range(2)]
    streams = [torch.cuda.Stream() for _ in range(2)]
    comm = torch.cuda.Stream()
    n_el = int(args.comm_mb * 1e6 / 4)
    src = torch.ones(n_el, dtype=torch.float32, device="cuda")
    dst = torch.empty_like(src)

    def run(with_comm, reserve):
        _lib.set_debug_knobs(grid_reserve=reserve or None)
        done = [None, None]
        torch.cuda.synchronize()
        t0 = torch.cuda.Event(enable_timing=True)
        t1 = torch.cuda.Event(enable_timing=True)
        t0.record(torch.cuda.current_stream())
        for s in streams + [comm]:
            s.wait_event(t0)
        for j in range(args.launches):
            k = j % 2
            if done[k] is not None:
                streams[k].wait_event(done[k])
            p = _lib.Params.from_buffer_copy(params)
            p.pass_ = (j * F) % 4096
            scene.render_passes_async(cam._state, p, F, outs[k].data_ptr(), streams[k].cuda_stream)
            ev = torch.cuda.Event()
            if with_comm:
                comm.wait_stream(streams[k])
                with torch.cuda.stream(comm):
                    torch.add(src, 1.0, out=dst)  # the stand-in collective: a kernel moving comm_mb
                ev.record(comm)
            else:
                ev.record(streams[k])
            done[k] = ev
        for s in streams + [comm]:
            torch.cuda.current_stream().wait_stream(s)
        t1.record(torch.cuda.current_stream())
        torch.cuda.synchronize()
        _lib.set_debug_knobs(grid_reserve=None)
        return t0.elapsed_time(t1) / (args.launches * F)

    cases = [("render only", False, 0)] + [(f"comm + reserve {r}" if r else "comm", True, r)
                                           for r in (int(x) for x in args.reserve.split(","))]
    res = {name: [] for name, _, _ in cases}
    run(False, 0)  # warm: contexts, candidate lists
    for _ in range(args.rounds):
        for name, c, r in cases:
            res[name].append(run(c, r))
    base = float(np.median(res["render only"]))
    for name, _, r in cases:
        med = float(np.median(res[name]))
        print(json.dumps({"config": args.config, "n": args.n, "rows": rows, "passes": F, "comm_mb": args.comm_mb,
                          "case": name, "reserve": r, "ms_per_frame": round(med, 4),
                          "vs_render_only": round(med / base, 4)}), flush=True)
    scene.release()


if __name__ == "__main__":
    main()
