#!/usr/bin/env python3
"""Diagnostic: how much of the traversal work belongs to primary (camera)
segments. Needs a -DTRAY_STATS_PRIMARY build (tools/build_variants.sh prim
"-DTRAY_STATS_PRIMARY").

    python tools/primary_share.py path/to/libtray_amd.so [--config c2]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib")
    ap.add_argument("--config", default="c2")
    args = ap.parse_args()
    import torch

    from bench import CONFIGS
    from tray_amd import _lib, ray

    label, seed, half, W, H, spp, depth = CONFIGS[args.config]
    spheres = ray.rich_scene_array(seed, half)
    cam = ray.RichSceneCamera()
    cam.Initialize(W, H)
    scene = _lib.DeviceScene(spheres, ray._background(ray.DefaultBackground()), 0, os.path.abspath(args.lib))
    params = _lib.make_params(W, H, depth, spp, 0.5, seed, output=_lib.OUT_RGB_F32)
    out = torch.empty((H, W, 3), dtype=torch.float32, device="cuda")
    stats = torch.zeros(8, dtype=torch.int64, device="cuda")
    scene.render_stats_async(cam._state, params, out.data_ptr(), stats.data_ptr(),
                             torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    names = ["segments", "sphere_tests", "box_tests", "nodes_primary", "leaves_primary", "boxes_primary",
             "nodes", "leaves"]
    d = dict(zip(names, stats.tolist()))
    samples = W * H * spp
    d["config"] = args.config
    d["segments_per_sample"] = round(d["segments"] / samples, 3)
    d["nodes_per_primary"] = round(d["nodes_primary"] / samples, 2)
    d["nodes_per_secondary"] = round((d["nodes"] - d["nodes_primary"]) / max(1, d["segments"] - samples), 2)
    d["leaves_per_primary"] = round(d["leaves_primary"] / samples, 2)
    d["leaves_per_secondary"] = round((d["leaves"] - d["leaves_primary"]) / max(1, d["segments"] - samples), 2)
    d["primary_share_nodes"] = round(d["nodes_primary"] / d["nodes"], 3)
    d["primary_share_leaves"] = round(d["leaves_primary"] / d["leaves"], 3)
    print(json.dumps(d))


if __name__ == "__main__":
    main()
