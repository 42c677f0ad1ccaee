#!/usr/bin/env python3
"""Strong-scaling rehearsal on ONE GPU: time each rank's row-tile shard of a
config (tile_rows / tile_count = N / tile_index = k, exactly what bench.py
--gpus N renders on rank k) and report, per N, the slowest shard and the
render-only scaling efficiency T(1) / (N * max_k T_k). The RCCL gather is not
included (bench.py adds it).

    python tools/shard_sim.py [--config c2] [--tile-rows 1] [--ns 1,2,4,8] [--reps 5]
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
    ap.add_argument("--tile-rows", type=int, default=1)
    ap.add_argument("--ns", default="1,2,4,8")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--frames-in-flight", type=int, default=1,
                    help="> 1: time --reps consecutive frames per shard overlapped this deep (bench.py's default is 3)")
    ap.add_argument("--passes", type=int, default=1,
                    help="frames per launch (tray_render_passes_async); times are per frame")
    ap.add_argument("--lib", default=None, help="a libtray_amd.so build to load (default: the in-tree one)")
    ap.add_argument("--knob", action="append", default=[], help="NAME=VALUE include/tray_debug.h knob (repeatable)")
    args = ap.parse_args()
    import numpy as np
    import torch

    from bench import CONFIGS
    from tray_amd import _lib, ray, shard

    label, seed, half, W, H, spp, depth = CONFIGS[args.config]
    spheres = ray.rich_scene_array(seed, half)
    cam = ray.RichSceneCamera()
    cam.Initialize(W, H)
    lib = os.path.abspath(args.lib) if args.lib else None
    if args.knob:
        _lib.set_debug_knobs(lib, **{k: int(v) for k, v in (kv.split("=", 1) for kv in args.knob)})
    scene = _lib.DeviceScene(spheres, ray._background(ray.DefaultBackground()), 0, *([lib] if lib else []))
    stream = torch.cuda.current_stream()
    base = _lib.make_params(W, H, depth, spp, 0.5, seed, output=_lib.OUT_RGB_F32)

    nslot = max(1, args.frames_in_flight)
    extra = [_lib.DeviceScene(spheres, ray._background(ray.DefaultBackground()), 0, *([lib] if lib else []))
             for _ in range(nslot - 1)]
    streams = [torch.cuda.Stream() for _ in range(nslot)]

    F = max(1, args.passes)

    def launch(sc, p, out, stream):
        if F == 1:
            sc.render_async(cam._state, p, out.data_ptr(), None, stream.cuda_stream)
        else:
            sc.render_passes_async(cam._state, p, F, out.data_ptr(), stream.cuda_stream)

    def time_pipelined(n, k):
        p = shard.shard_params(base, args.tile_rows, n, k)
        outs = [torch.empty((F, _lib.params_rows(p), W, 3), dtype=torch.float32, device="cuda") for _ in range(nslot)]
        scs = [scene] + extra
        for i in range(nslot):  # warm
            launch(scs[i], p, outs[i], streams[i])
        torch.cuda.synchronize()
        reps = max(args.reps, 4 * nslot)
        a = torch.cuda.Event(enable_timing=True)
        a.record(torch.cuda.current_stream())
        for s_ in streams:
            s_.wait_event(a)
        for i in range(reps):
            j = i % nslot
            launch(scs[j], p, outs[j], streams[j])
        ends = []
        for s_ in streams:
            e = torch.cuda.Event(enable_timing=True)
            e.record(s_)
            ends.append(e)
        torch.cuda.synchronize()
        return max(a.elapsed_time(e) for e in ends) / (reps * F)

    def time_shard(n, k):
        if nslot > 1 or F > 1:
            return time_pipelined(n, k)
        p = shard.shard_params(base, args.tile_rows, n, k)
        out = torch.empty((_lib.params_rows(p), W, 3), dtype=torch.float32, device="cuda")
        scene.render_async(cam._state, p, out.data_ptr(), None, stream.cuda_stream)  # warm
        ts = []
        for _ in range(args.reps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(stream)
            scene.render_async(cam._state, p, out.data_ptr(), None, stream.cuda_stream)
            b.record(stream)
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b))
        return float(np.median(ts))

    t1 = None
    for n in [int(x) for x in args.ns.split(",")]:
        times = [time_shard(n, k) for k in range(n)]
        if n == 1:
            t1 = times[0]
        rec = {"config": args.config, "n": n, "tile_rows": args.tile_rows, "frames_in_flight": nslot, "passes": F, "max_ms": round(max(times), 4),
               "min_ms": round(min(times), 4), "mean_ms": round(float(np.mean(times)), 4)}
        if t1:
            rec["render_efficiency"] = round(t1 / (n * max(times)), 4)
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
