#!/usr/bin/env python3
"""Instruction-mix summary of tools/profile_counters*.sh passes: per counter, the
median over the timed (non-instrumented) render_kernel launches.

    python tools/pmc_mix.py gpurun_out/ev8/all --label "C2, v8" > profiles/r1_pmc_mix_v8.json
"""
import argparse
import csv
import glob
import json
import os
import statistics
import sys


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root", help="gpu_profile_all.sh output dir (holds pmc1/, pmc2/)")
    ap.add_argument("--label", default="")
    ap.add_argument("--frames", type=int, default=16, help="frames per launch of the profiled bench command")
    ap.add_argument("--config", default="c2", help="bench config: picks the kernel instance (how r is summed)")
    a = ap.parse_args()
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from bench import CONFIGS

    spp = CONFIGS[a.config][5]
    # kAcc: 1 on-chip sums per 64-sample chunk (64 | r), 2 per pixel-pass (r = 16, 32), 0 none
    want = f", true, false, false, false, {1 if spp % 64 == 0 else 2 if spp in (16, 32) else 0}, "
    vals, kernel = {}, None
    for f in sorted(glob.glob(os.path.join(a.root, "pmc*", "p*", "*counter_collection.csv"))):
        per = {}
        for row in csv.DictReader(open(f)):
            name = row["Kernel_Name"]
            # the timed kernel: render_kernel<mode, true, false (no stats), spill>
            # the timed BVH kernel: render_kernel<layout, true, false (no stats), false (no spill), false, kAcc (on-chip sums), S (node steps)>
            # (layout 1 for the book cover, 2 for the dense C5 scene)
            if "render_kernel<" not in name or want not in name:
                continue
            kernel = name
            key = (row["Counter_Name"], row["Dispatch_Id"])
            per[key] = per.get(key, 0.0) + float(row["Counter_Value"])
        for (c, _), v in per.items():
            vals.setdefault(c, []).append(v)
    counters = {c: statistics.median(v) for c, v in sorted(vals.items())}
    busy = counters.get("SQ_ACTIVE_INST_VALU")
    hashes = {open(h).read().strip() for h in glob.glob(os.path.join(a.root, "pmc*", "code_object_sha256.txt"))}
    if len(hashes) > 1:
        raise SystemExit(f"counter passes measured different device code: {sorted(hashes)}")
    out = {"kernel": kernel, "label": a.label, "frames_per_launch": a.frames,
           "code_object_sha256": hashes.pop() if hashes else None,
           "method": "tools/profile_counters.sh + profile_counters2.sh, --frames-in-flight 1, median over launches",
           "counters": counters}
    if busy and counters.get("SQ_THREAD_CYCLES_VALU"):
        # active lanes per issued VALU instruction
        out["valu_lane_utilisation"] = round(counters["SQ_THREAD_CYCLES_VALU"] / (64 * busy), 3)
    fp64 = sum(counters.get(c, 0.0) for c in ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64",
                                               "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_TRANS_F64"))
    valu, gui = counters.get("SQ_INSTS_VALU"), counters.get("GRBM_GUI_ACTIVE")
    if valu and gui and fp64:
        # issue cycles of the VALU instructions (a wave64 FP64 op holds a SIMD-32 for 4 cycles,
        # any other VALU op for 2: MI355X_MICROARCH.md) over the SIMD-cycles of the launch
        # (256 CUs x 4 SIMDs; GRBM_GUI_ACTIVE sums the 8 XCDs' busy cycles)
        out["valu_issue_utilisation"] = round((4 * fp64 + 2 * (valu - fp64)) / (1024 * gui / 8), 3)
        out["fp64_share_of_valu"] = round(fp64 / valu, 3)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
