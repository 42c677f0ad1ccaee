#!/usr/bin/env python3
"""Where does the 8-way shard lose its ~3 %? The same amount of
work two ways, alternating in one process, for rocprofv3 --pmc passes:

  A: rank 0's rows of an N-way 1-row interleaved split, 16 progressive passes
     in one launch (what each rank of `bench.py --gpus N` launches);
  B: the whole frame, 16/N passes in one launch (the same number of samples).

    rocprofv3 --pmc <counters> --kernel-include-regex render_kernel -d OUT -o pmc --output-format csv \\
        -- python3 tools/shard_pmc.py --n 8 --reps 6
    python tools/shard_pmc.py --summarize OUT_1 OUT_2 ...      (per-counter medians of A and B)

Without a profiler it prints the HIP-event times of A and B.
"""
import argparse
import csv
import glob
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(args):
    import torch

    from bench import CONFIGS
    from tray_amd import _lib, ray, shard

    _, seed, half, W, H, spp, depth = CONFIGS[args.config]
    spp = args.spp or spp
    spheres = ray.rich_scene_array(seed, half)
    cam = ray.RichSceneCamera()
    cam.Initialize(W, H)
    bg = ray._background(ray.DefaultBackground())
    base = _lib.make_params(W, H, depth, spp, 0.5, seed, output=_lib.OUT_RGB_F32)
    pa = shard.shard_params(base, args.tile_rows, args.n, args.rank)
    if args.force_tiles:  # the tiled code path even for n = 1 (row_of's per-item division)
        pa = _lib.Params.from_buffer_copy(base)
        pa.tile_rows, pa.tile_count, pa.tile_index = args.tile_rows, args.n, 0
    for kv in args.knob:
        name, value = kv.split("=")
        _lib.set_debug_knobs(args.lib, **{name: int(value)})
    fa, fb = args.passes, max(1, args.passes // args.n)
    scenes = [_lib.DeviceScene(spheres, bg, 0, args.lib) for _ in range(2)]  # own work queue and buffers each
    oa = torch.empty((fa, _lib.params_rows(pa), W, 3), dtype=torch.float32, device="cuda")
    ob = torch.empty((fb, H, W, 3), dtype=torch.float32, device="cuda")
    stream = torch.cuda.current_stream()
    times = {"A": [], "B": []}
    for r in range(args.reps + 1):
        for name, sc, p, n, out in (("A", scenes[0], pa, fa, oa), ("B", scenes[1], base, fb, ob)):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            sc.render_passes_async(cam._state, p, n, out.data_ptr(), stream.cuda_stream)
            e1.record(stream)
            torch.cuda.synchronize()
            if r:
                times[name].append(e0.elapsed_time(e1))
    samples = {"A": _lib.params_rows(pa) * W * spp * fa, "B": H * W * spp * fb}
    print(json.dumps({"config": args.config, "lib": args.lib, "n": args.n, "tile_rows": args.tile_rows, "knobs": args.knob, "force_tiles": args.force_tiles, "rank": args.rank, "spp": spp, "A": {"passes": fa, "samples": samples["A"],
                                                                  "median_ms": statistics.median(times["A"])},
                      "B": {"passes": fb, "samples": samples["B"], "median_ms": statistics.median(times["B"])},
                      "A_over_B_per_sample": round(statistics.median(times["A"]) / samples["A"] /
                                                   (statistics.median(times["B"]) / samples["B"]), 4)}))
    for s in scenes:
        s.release()


def summarize(dirs):
    """Per counter: median over A dispatches and over B dispatches (they alternate A, B, ...;
    the first pair is warm-up)."""
    vals = {}
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            per = {}
            for row in csv.DictReader(open(f)):
                if "render_kernel<" not in row["Kernel_Name"]:
                    continue
                key = (row["Counter_Name"], int(row["Dispatch_Id"]))
                per[key] = per.get(key, 0.0) + float(row["Counter_Value"])
            ids = sorted({k[1] for k in per})
            for c in sorted({k[0] for k in per}):
                seq = [per[(c, i)] for i in ids if (c, i) in per]
                a, b = seq[2::2], seq[3::2]  # skip the warm-up pair
                if a and b:
                    vals[c] = {"A": statistics.median(a), "B": statistics.median(b),
                               "A_over_B": round(statistics.median(a) / statistics.median(b), 4)}
    print(json.dumps(vals, indent=1))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--n", type=int, default=8)
    ap.add_argument("--passes", type=int, default=16, help="passes of A (B renders passes / n)")
    ap.add_argument("--tile-rows", type=int, default=1)
    ap.add_argument("--lib", default=None, help="another build of libtray_amd.so (tools/build_variants.sh)")
    ap.add_argument("--force-tiles", action="store_true")
    ap.add_argument("--rank", type=int, default=0, help="which shard A renders")
    ap.add_argument("--spp", type=int, default=0, help="override rays per pixel")
    ap.add_argument("--knob", action="append", default=[], help="tray_debug.h knob NAME=VALUE (both A and B)")
    ap.add_argument("--reps", type=int, default=6)
    ap.add_argument("--summarize", nargs="*")
    args = ap.parse_args()
    if args.summarize:
        summarize(args.summarize)
    else:
        run(args)


if __name__ == "__main__":
    main()
