#!/usr/bin/env python3
"""Where the drop-in call's time over the kernel goes:
bench.py's `e2e_ms` (one synchronous tray_render of the C2 frame into host
memory as RGBA8, the call a Go Render makes) against its parts, same process,
same scene, medians of --reps:

  e2e_ms            tray_render into pageable host memory (what bench.py reports)
  launch_host_ms    tray_render_async into a device buffer + stream sync, host-timed
  launch_event_ms   the same launch between two HIP events (kernel + resolve only)
  d2h_pageable_ms   hipMemcpy of the RGBA8 frame (3.7 MB) into pageable host memory
  d2h_pinned_ms     the same into pinned host memory

    python tools/e2e_split.py [--config c2] [--reps 7] [--knob work_order=0]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--reps", type=int, default=7)
    ap.add_argument("--knob", action="append", default=[], help="NAME=VALUE include/tray_debug.h knob (repeatable)")
    args = ap.parse_args()
    import numpy as np
    import torch

    from bench import CONFIGS
    from tray_amd import _lib, ray

    if args.knob:
        _lib.set_debug_knobs(None, **{k: int(v) for k, v in (kv.split("=", 1) for kv in args.knob)})

    _, seed, half, W, H, spp, depth = CONFIGS[args.config]
    spheres = ray.rich_scene_array(seed, half)
    cam = ray.RichSceneCamera()
    cam.Initialize(W, H)
    bg = ray._background(ray.DefaultBackground())
    p = _lib.make_params(W, H, depth, spp, 0.5, seed, output=_lib.OUT_RGBA8)
    for _ in range(2):
        _lib.render(spheres, bg, cam._state, p)  # warm: upload, buffers, queues

    def med(f):
        ts = []
        for _ in range(args.reps):
            t0 = time.perf_counter()
            f()
            ts.append((time.perf_counter() - t0) * 1e3)
        return round(float(np.median(ts)), 4)

    rec = {"config": args.config, "knobs": args.knob, "e2e_ms": med(lambda: _lib.render(spheres, bg, cam._state, p))}
    dev = _lib.DeviceScene(spheres, bg, 0)
    out = torch.empty((H, W, 4), dtype=torch.uint8, device="cuda")
    stream = torch.cuda.current_stream()

    def launch():
        dev.render_async(cam._state, p, out.data_ptr(), None, stream.cuda_stream)
        torch.cuda.synchronize()
    launch()
    rec["launch_host_ms"] = med(launch)
    ev = []
    for _ in range(args.reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        dev.render_async(cam._state, p, out.data_ptr(), None, stream.cuda_stream)
        b.record(stream)
        torch.cuda.synchronize()
        ev.append(a.elapsed_time(b))
    rec["launch_event_ms"] = round(float(np.median(ev)), 4)
    host = torch.from_numpy(np.empty((H, W, 4), dtype=np.uint8))  # pageable, like a Go []byte
    pinned = torch.empty((H, W, 4), dtype=torch.uint8).pin_memory()
    rec["d2h_pageable_ms"] = med(lambda: host.copy_(out))
    rec["d2h_pinned_ms"] = med(lambda: (pinned.copy_(out, non_blocking=True), torch.cuda.synchronize()))
    rec["frame_bytes"] = W * H * 4
    rec["gap_ms"] = round(rec["e2e_ms"] - rec["launch_event_ms"], 4)
    dev.release()
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
