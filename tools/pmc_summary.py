#!/usr/bin/env python3
"""Turn a tools/profile_bench.sh output directory into profiles/pmc_<config>.json
(the `roofline.traffic` bench.py reports) and copy the rocprofv3 summaries into
profiles/ under a round tag.

    python tools/pmc_summary.py gpurun_out/prof_c2 --config c2 --tag r1_c2_v5

HBM bytes per launch follow MI355X_MICROARCH.md's HBM section: FETCH_SIZE (KB)
x 1024 x 2 on gfx950, WRITE_SIZE (KB) x 1024, each from its own --pmc pass; the
value is the median over the timed (non-instrumented) megakernel launches.
"""
import argparse
import csv
import json
import os
import shutil
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# The timed BVH kernel, any LDS layout (1: book cover, 2: dense C5) and step count:
# render_kernel<L, bvh, stats, progress, spill, kAcc, S>, kAcc the on-chip accumulation:
# 1 per 64-sample chunk (64 | r: C2-C5), 2 per pixel-pass (r = 16, 32: C1), 0 none.
KERNELS = {k: f", true, false, false, false, {k}, " for k in (0, 1, 2)}
KERNEL = KERNELS[1]


ACC_WHAT = {1: "on-chip accumulation, one record per 64-sample chunk",
            2: "on-chip accumulation, one record per pixel-pass", 0: "per-sample buffer"}


def acc_mode(spp):
    return 1 if spp % 64 == 0 else 2 if spp in (16, 32) else 0


def values(path):
    rows = [r for r in csv.DictReader(open(path)) if "tray::render_kernel<" in r["Kernel_Name"] and
            KERNEL in r["Kernel_Name"]]
    # drop the first launches of each slot: their buffers are cold (first touch)
    vals = [float(r["Counter_Value"]) for r in rows]
    return vals[len(vals) // 3:] if len(vals) >= 3 else vals


def code_hash(d):
    """The device-code hash the profiling run recorded (profile_*.sh), else the in-tree build's."""
    for p in (os.path.join(d, "code_object_sha256.txt"), os.path.join(os.path.dirname(d), "code_object_sha256.txt")):
        if os.path.exists(p):
            return open(p).read().strip()
    sys.path.insert(0, ROOT)
    from tray_amd import _lib

    return _lib.code_object_sha256()


def main():
    global KERNEL
    ap = argparse.ArgumentParser()
    ap.add_argument("profdir")
    ap.add_argument("--config", default="c2")
    ap.add_argument("--tag", required=True)
    ap.add_argument("--frames", type=int, default=16, help="frames per launch of the profiled bench command")
    args = ap.parse_args()
    d = args.profdir
    # A launch of F frames runs in bands (tray_kernel.hip band_tile_rows), one megakernel
    # dispatch each, and the counters are per dispatch: C2 is one band per 16-frame launch,
    # C3/C5 several. With on-chip sums (C1-C5) a band holds up to
    # 2^31 samples, else 2^30 (tray_kernel.hpp kMaxBandSamplesAcc / kMaxBandSamples).
    sys.path.insert(0, ROOT)
    from bench import CONFIGS

    _, _, _, W, H, spp, _ = CONFIGS[args.config]
    tiles_x = (W + 7) // 8
    limit = 1 << (31 if acc_mode(spp) else 30)
    KERNEL = KERNELS[acc_mode(spp)]
    fetch_kb = statistics.median(values(os.path.join(d, "FETCH_SIZE", "pmc_counter_collection.csv")))
    write_kb = statistics.median(values(os.path.join(d, "WRITE_SIZE", "pmc_counter_collection.csv")))
    band_rows = 8 * max(1, limit // (tiles_x * 64 * spp * args.frames))
    bands = -(-H // band_rows)
    fetch = fetch_kb * 1024 * 2 * bands
    write = write_kb * 1024 * bands
    copies = {
        os.path.join(d, "kt", "kt_kernel_stats.csv"): f"{args.tag}_kernel_stats.csv",
        os.path.join(d, "FETCH_SIZE", "pmc_counter_collection.csv"): f"{args.tag}_pmc_fetch_size.csv",
        os.path.join(d, "WRITE_SIZE", "pmc_counter_collection.csv"): f"{args.tag}_pmc_write_size.csv",
    }
    for src, dst in copies.items():
        shutil.copy(src, os.path.join(ROOT, "profiles", dst))
    rec = {
        "config": args.config,
        "code_object_sha256": code_hash(d),
        "frames_per_launch": args.frames,
        "kernel": f"tray::render_kernel<L, true, false, false, false, {acc_mode(spp)}, S> (BVH, LDS layout L, "
                  f"no stack spill, {ACC_WHAT[acc_mode(spp)]}, S node steps)",
        "bands_per_launch": bands,
        "FETCH_SIZE_KB_raw_per_dispatch": fetch_kb,
        "WRITE_SIZE_KB_per_dispatch": write_kb,
        "fetch_bytes_corrected": fetch,
        "write_bytes": write,
        "hbm_bytes_per_launch": int(fetch + write),
        "note": "megakernel only, per launch (frames_per_launch frames). With on-chip accumulation it writes one "
                "32-B record of fixed-point sums per 64-sample chunk (64 | r) or per pixel-pass (r = 16, 32) and "
                "reads the primary-ray "
                "candidate records (16 B per pixel per frame); without it, one 24-B colour per sample. The "
                "resolve kernel reads the records back and writes the frames.",
        "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes (MI355X_MICROARCH.md HBM "
                  "section: FETCH_SIZE x2 on gfx950, WRITE_SIZE exact); median over the warm dispatches x "
                  "bands_per_launch",
        "source": [f"profiles/{v}" for v in list(copies.values())[1:]],
    }
    with open(os.path.join(ROOT, "profiles", f"pmc_{args.config}.json"), "w") as f:
        json.dump(rec, f, indent=1)
    print(json.dumps(rec, indent=1))


if __name__ == "__main__":
    main()
