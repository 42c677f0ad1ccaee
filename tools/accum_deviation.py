#!/usr/bin/env python3
"""Observed colour deviation of the two pixel-sum modes from the oracle (Go's FP64
sum in sample order, oracle/tray_oracle.c), on the same seeded region of a
benchmark scene: the fixed-point sums (default for 64 | r) and the FP64 sum in
sample order (TRAY_FLAG_ORDERED_SUM). Prints one JSON line per config.

    python tools/accum_deviation.py [--w 96 --h 54]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--w", type=int, default=96)
    ap.add_argument("--h", type=int, default=54)
    args = ap.parse_args()
    import numpy as np

    from bench import CONFIGS
    from oracle import oracle as O
    from tray_amd import _lib as L, ray

    for c in ("c2", "c5"):
        _, seed, half, _, _, spp, depth = CONFIGS[c]
        spheres = ray.rich_scene_array(seed, half)
        cam = ray.RichSceneCamera()
        cam.Initialize(args.w, args.h)
        bg = ray._background(ray.DefaultBackground())
        bg_arr = np.array(list(bg.color_a) + list(bg.color_b))
        p = L.make_params(args.w, args.h, depth, spp, 0.5, seed)
        fixed, seg = L.render(spheres, bg, cam._state, p, 0, segments=True)
        po = L.make_params(args.w, args.h, depth, spp, 0.5, seed, flags=L.FLAG_ORDERED_SUM)
        f64, seg2 = L.render(spheres, bg, cam._state, po, 0, segments=True)
        ref, rseg = O.render(spheres, bg_arr, cam._state.as_array(), args.w, args.h, spp, depth, 0.5, seed,
                             workers=min(16, os.cpu_count() or 4))
        print(json.dumps({
            "config": c, "region": f"{args.w}x{args.h}", "rays_per_pixel": spp, "max_depth": depth,
            "paths_equal": bool(np.array_equal(seg, rseg) and np.array_equal(seg2, rseg)),
            "fixed_vs_oracle_linf": float(np.max(np.abs(fixed - ref))),
            "fp64_order_vs_oracle_linf": float(np.max(np.abs(f64 - ref))),
            "fixed_vs_fp64_order_linf": float(np.max(np.abs(fixed - f64))),
            "fixed_bits_equal_oracle_share": float(np.mean(fixed == ref)),
            "fp64_order_bits_equal_oracle_share": float(np.mean(f64 == ref)),
        }), flush=True)


if __name__ == "__main__":
    main()
