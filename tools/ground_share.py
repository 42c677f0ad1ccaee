#!/usr/bin/env python3
"""Diagnostic: how much traversal work belongs to segments that leave an
out-of-tree sphere (the ground) upward (direction on the +y cube face) or in any
direction. Needs a -DTRAY_STATS_GROUND build (tools/build_variants.sh ground
"-DTRAY_STATS_GROUND").

    python tools/ground_share.py path/to/libtray_amd.so [--config c2]
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
    stats = torch.zeros(11, dtype=torch.int64, device="cuda")
    scene.render_stats_async(cam._state, params, out.data_ptr(), stats.data_ptr(),
                             torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    v = stats.tolist()
    names = ["segments", "sphere_tests", "box_tests", "seg_ground_up", "seg_ground_any", "nodes_ground_up",
             "nodes_ground_any", "leaves_ground_up", "leaves_ground_any", "nodes", "leaves"]
    d = dict(zip(names, v))
    d["config"] = args.config
    d["share_segments_ground_up"] = round(d["seg_ground_up"] / d["segments"], 3)
    d["share_segments_ground_any"] = round(d["seg_ground_any"] / d["segments"], 3)
    d["share_nodes_ground_up"] = round(d["nodes_ground_up"] / max(1, d["nodes"]), 3)
    d["share_nodes_ground_any"] = round(d["nodes_ground_any"] / max(1, d["nodes"]), 3)
    d["share_leaves_ground_up"] = round(d["leaves_ground_up"] / max(1, d["leaves"]), 3)
    d["nodes_per_ground_up"] = round(d["nodes_ground_up"] / max(1, d["seg_ground_up"]), 2)
    d["nodes_per_other"] = round((d["nodes"] - d["nodes_ground_up"]) / max(1, d["segments"] - d["seg_ground_up"]), 2)
    print(json.dumps(d))


if __name__ == "__main__":
    main()
