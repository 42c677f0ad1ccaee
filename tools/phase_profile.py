#!/usr/bin/env python3
"""Diagnostic: per-phase cycle split of the BVH kernel from a -DTRAY_PROFILE
build (tools/build_variants.sh prof "-DTRAY_PROFILE"). Not a timing tool: the
stamps serialise phases; read the SHARES.

    python tools/phase_profile.py path/to/libtray_amd.so [--config c2]
"""
import argparse
import json
import os
import sys

PHASES = ("cyc_refill", "cyc_node", "cyc_leaf", "cyc_shade")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib")
    ap.add_argument("--config", default="c2")
    ap.add_argument("--shard", default=None, help="N,K: rank K's row tiles of an N-way split (1-row tiles)")
    ap.add_argument("--refill-split", action="store_true", help="the library is a -DTRAY_PROFILE_REFILL build")
    ap.add_argument("--waves", type=int, default=256 * 16, help="waves in the launch (CUs x waves per CU)")
    ap.add_argument("--material", action="store_true",
                    help="the library is a -DTRAY_PROFILE_MATERIAL build: report the shading divergence census")
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
    if args.shard:
        from tray_amd import shard
        n, k = (int(v) for v in args.shard.split(","))
        params = shard.shard_params(params, 1, n, k)
    out = torch.empty((_lib.params_rows(params), W, 3), dtype=torch.float32, device="cuda")
    stats = torch.zeros(32 + 2 * args.waves + 64, dtype=torch.int64, device="cuda")
    scene.render_stats_async(cam._state, params, out.data_ptr(), stats.data_ptr(),
                             torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    allv = stats.tolist()
    v = allv[:22]
    # -DTRAY_PROFILE_REFILL: stats[13], [16], [17], [18] (slots 10, 13-15) hold the refill split
    refill_split = dict(zip(["refill_assign", "refill_camera", "refill_hit", "refill_shade"],
                            [allv[13], allv[16], allv[17], allv[18]]))
    se = allv[32:32 + 2 * args.waves]
    names = ["segments", "sphere_tests", "box_tests", "cyc_refill", "cyc_node", "cyc_leaf", "cyc_shade",
             "node_iters", "node_lanes", "leaf_phases", "leaf_lanes", "shade_phases", "shade_lanes", "loop_iters", "node_leafwait_lanes", "node_shadewait_lanes", "refill_phases", "refill_lanes",
             "unused_15", "rt_end_max", "rt_life_sum",
             "rt_start_min_inv"]
    d = dict(zip(names, v))
    if args.refill_split:
        d["refill_split_share"] = {k: round(x / max(1, d["cyc_refill"]), 3) for k, x in refill_split.items()}
    cyc = sum(d[k] for k in PHASES)
    d["share"] = {k: round(d[k] / cyc, 3) for k in PHASES}
    d["lanes_per_node_iter"] = round(d["node_lanes"] / max(1, d["node_iters"]), 1)
    d["leafwait_lanes_per_node_iter"] = round(d["node_leafwait_lanes"] / max(1, d["node_iters"]), 1)
    d["shadewait_lanes_per_node_iter"] = round(d["node_shadewait_lanes"] / max(1, d["node_iters"]), 1)
    d["lanes_per_leaf_phase"] = round(d["leaf_lanes"] / max(1, d["leaf_phases"]), 1)
    d["lanes_per_shade_phase"] = round(d["shade_lanes"] / max(1, d["shade_phases"]), 1)
    d["lanes_per_refill_phase"] = round(d["refill_lanes"] / max(1, d["refill_phases"]), 1)
    d["cyc_per_refill_phase"] = round(d["cyc_refill"] / max(1, d["refill_phases"]), 1)
    d["cyc_per_node_iter"] = round(d["cyc_node"] / max(1, d["node_iters"]), 1)
    d["cyc_per_leaf_phase"] = round(d["cyc_leaf"] / max(1, d["leaf_phases"]), 1)
    d["cyc_per_shade_phase"] = round(d["cyc_shade"] / max(1, d["shade_phases"]), 1)
    # Tail: kernel span (latest exit - earliest start) vs the mean wave lifetime,
    # on the 100 MHz constant-rate clock (s_memrealtime).
    start_min = (1 << 64) - 1 - (d["rt_start_min_inv"] % (1 << 64))
    waves = args.waves
    span = d["rt_end_max"] - start_min
    d["span_us"] = round(span / 100.0, 1)
    d["mean_wave_life_us"] = round(d["rt_life_sum"] / waves / 100.0, 1)
    d["tail_idle_frac"] = round(1.0 - d["rt_life_sum"] / waves / max(1, span), 4)
    import numpy as np
    st_ = np.array(se[0::2], dtype=np.float64)
    en_ = np.array(se[1::2], dtype=np.float64)
    ok = en_ > 0
    st_, en_ = st_[ok] - start_min, en_[ok] - start_min
    q = [0, 1, 10, 50, 90, 99, 100]
    d["waves_seen"] = int(ok.sum())
    d["wave_start_us_pct"] = {str(k): round(float(np.percentile(st_, k)) / 100.0, 1) for k in q}
    d["wave_end_us_pct"] = {str(k): round(float(np.percentile(en_, k)) / 100.0, 1) for k in q}
    if args.material:
        cls = ["miss", "last", "lambertian", "metal0", "metal_fuzz", "dielectric"]
        mat = allv[32 + 2 * args.waves:]
        for site, name in enumerate(["refill_shade", "shade"]):
            c = mat[18 * site: 18 * site + 18]
            passes = max(1, c[16])
            d["material_" + name] = {
                "passes": c[16], "lanes": c[17], "lanes_per_pass": round(c[17] / passes, 2),
                "passes_with": {k: round(c[i] / passes, 4) for i, k in enumerate(cls)},
                "lanes_of": {k: c[6 + i] for i, k in enumerate(cls)},
                "lanes_per_pass_with": {k: round(c[6 + i] / max(1, c[i]), 2) for i, k in enumerate(cls)},
                "bodies_per_pass": {str(b): round(c[12 + b] / passes, 4) for b in range(4)},
            }
    print(json.dumps(d))


if __name__ == "__main__":
    main()
