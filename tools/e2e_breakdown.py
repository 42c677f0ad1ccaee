#!/usr/bin/env python3
"""Where the cold synchronous render's extra time goes (C2): scene upload
(BVH build + copies), the first render of a fresh scene (sample-buffer
allocation), a warm render, and the host copy. Diagnostic only.

    python tools/e2e_breakdown.py
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    from bench import CONFIGS
    from tray_amd import _lib, ray

    _, seed, half, W, H, spp, depth = CONFIGS["c2"]
    spheres = ray.rich_scene_array(seed, half)
    cam = ray.RichSceneCamera()
    cam.Initialize(W, H)
    bg = ray._background(ray.DefaultBackground())
    p = _lib.make_params(W, H, depth, spp, 0.5, seed, output=_lib.OUT_RGBA8)
    out = torch.empty((H, W, 4), dtype=torch.uint8, device="cuda")
    warm = _lib.DeviceScene(spheres, bg, 0)  # loads the code object, first launch
    warm.render_async(cam._state, p, out.data_ptr())
    torch.cuda.synchronize()
    rec = {}
    t0 = time.perf_counter()
    sc = _lib.DeviceScene(spheres, bg, 0)
    rec["scene_upload_ms"] = (time.perf_counter() - t0) * 1e3
    t0 = time.perf_counter()
    sc.render_async(cam._state, p, out.data_ptr())
    torch.cuda.synchronize()
    rec["first_render_ms"] = (time.perf_counter() - t0) * 1e3
    t0 = time.perf_counter()
    sc.render_async(cam._state, p, out.data_ptr())
    torch.cuda.synchronize()
    rec["warm_render_ms"] = (time.perf_counter() - t0) * 1e3
    t0 = time.perf_counter()
    host = out.cpu()
    rec["d2h_pageable_ms"] = (time.perf_counter() - t0) * 1e3
    for k in range(3):
        t0 = time.perf_counter()
        _lib.render(spheres, bg, cam._state, p)
        rec[f"tray_render_{k}_ms"] = (time.perf_counter() - t0) * 1e3
    print(json.dumps({k: round(v, 3) for k, v in rec.items()}))
    del host


if __name__ == "__main__":
    main()
