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

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNEL = "tray::render_kernel<1, true, false, false, false>"


def values(path):
    rows = [r for r in csv.DictReader(open(path)) if KERNEL in r["Kernel_Name"]]
    # drop the first launches of each slot: their buffers are cold (first touch)
    vals = [float(r["Counter_Value"]) for r in rows]
    return vals[len(vals) // 3:] if len(vals) >= 3 else vals


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("profdir")
    ap.add_argument("--config", default="c2")
    ap.add_argument("--tag", required=True)
    ap.add_argument("--frames", type=int, default=16, help="frames per launch of the profiled bench command")
    args = ap.parse_args()
    d = args.profdir
    fetch_kb = statistics.median(values(os.path.join(d, "FETCH_SIZE", "pmc_counter_collection.csv")))
    write_kb = statistics.median(values(os.path.join(d, "WRITE_SIZE", "pmc_counter_collection.csv")))
    fetch = fetch_kb * 1024 * 2
    write = write_kb * 1024
    copies = {
        os.path.join(d, "kt", "kt_kernel_stats.csv"): f"{args.tag}_kernel_stats.csv",
        os.path.join(d, "FETCH_SIZE", "pmc_counter_collection.csv"): f"{args.tag}_pmc_fetch_size.csv",
        os.path.join(d, "WRITE_SIZE", "pmc_counter_collection.csv"): f"{args.tag}_pmc_write_size.csv",
    }
    for src, dst in copies.items():
        shutil.copy(src, os.path.join(ROOT, "profiles", dst))
    rec = {
        "config": args.config,
        "frames_per_launch": args.frames,
        "kernel": "tray::render_kernel<1, true, false, false, false> (BVH, whole scene in LDS, no stack spill)",
        "FETCH_SIZE_KB_raw": fetch_kb,
        "WRITE_SIZE_KB": write_kb,
        "fetch_bytes_corrected": fetch,
        "write_bytes": write,
        "hbm_bytes_per_launch": int(fetch + write),
        "note": "megakernel only, per launch (frames_per_launch frames); its HBM traffic is the per-sample "
                "colour buffer (24 B/sample). The resolve kernel reads it back.",
        "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes (MI355X_MICROARCH.md HBM "
                  "section: FETCH_SIZE x2 on gfx950, WRITE_SIZE exact); median over the warm launches",
        "source": [f"profiles/{v}" for v in list(copies.values())[1:]],
    }
    with open(os.path.join(ROOT, "profiles", f"pmc_{args.config}.json"), "w") as f:
        json.dump(rec, f, indent=1)
    print(json.dumps(rec, indent=1))


if __name__ == "__main__":
    main()
