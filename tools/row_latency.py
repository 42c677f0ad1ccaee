#!/usr/bin/env python3
"""Latency probe: render single rows (or short row ranges) of a config, where
every lane gets at most one sample, so the launch time is the slowest path of
those rows plus launch overhead. Prints per-range kernel ms and the range's
max / mean segments per sample.

    python tools/row_latency.py [--config c2] [--rows 0,100,360,600] [--count 1]
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
    ap.add_argument("--rows", default="0,100,300,360,420,600,700")
    ap.add_argument("--count", type=int, default=1)
    ap.add_argument("--depths", default=None, help="comma list of max depths to sweep (default: the config's)")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--lib", default=None, help="a libtray_amd.so build to load (default: the in-tree one)")
    args = ap.parse_args()
    import numpy as np
    import torch

    from bench import CONFIGS
    from tray_amd import _lib, ray

    label, seed, half, W, H, spp, depth = CONFIGS[args.config]
    spheres = ray.rich_scene_array(seed, half)
    cam = ray.RichSceneCamera()
    cam.Initialize(W, H)
    lib = os.path.abspath(args.lib) if args.lib else None
    scene = _lib.DeviceScene(spheres, ray._background(ray.DefaultBackground()), 0, *([lib] if lib else []))
    stream = torch.cuda.current_stream()
    depths = [int(v) for v in args.depths.split(",")] if args.depths else [depth]
    for y0, depth in [(y, d) for y in (int(v) for v in args.rows.split(",")) for d in depths]:
        p = _lib.make_params(W, H, depth, spp, 0.5, seed, y_start=y0, y_end=y0 + args.count,
                             output=_lib.OUT_RGB_F32)
        out = torch.empty((args.count, W, 3), dtype=torch.float32, device="cuda")
        seg = torch.zeros((args.count, W), dtype=torch.int32, device="cuda")
        scene.render_async(cam._state, p, out.data_ptr(), seg.data_ptr(), stream.cuda_stream)
        torch.cuda.synchronize()
        ts = []
        for _ in range(args.reps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(stream)
            scene.render_async(cam._state, p, out.data_ptr(), None, stream.cuda_stream)
            b.record(stream)
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b))
        s = seg.cpu().numpy().astype(np.float64) / spp
        print(json.dumps({"y0": y0, "rows": args.count, "depth": depth, "ms": round(float(np.median(ts)), 4),
                          "seg_per_sample_mean": round(float(s.mean()), 3),
                          "pixel_mean_seg_max": round(float(s.max()), 3)}), flush=True)


if __name__ == "__main__":
    main()
