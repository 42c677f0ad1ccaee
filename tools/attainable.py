#!/usr/bin/env python3
"""Attainable-bound analysis of the megakernel's FP64-roof fraction (bench.py
roofline.frac): how much of the gap to 1.0 the parity contract fixes (the
instruction stream itself: correctly rounded sqrt / division sequences,
Philox, the FP32 slab tests, compares, selects and moves around them) and how
much SIMT divergence (inactive lanes) and issue stalls cost.

From a pmc_mix record (tools/pmc_mix.py: SQ_INSTS_VALU and its FP64 classes,
SQ_THREAD_CYCLES_VALU / SQ_ACTIVE_INST_VALU, GRBM_GUI_ACTIVE) and the bench
line's roofline record (frac, the ops model):

  issue_util  = VALU issue cycles (4 per FP64, 2 per other wave64 VALU
                instruction, MI355X_MICROARCH.md) / the launch's SIMD-cycles
  lane_util   = active lanes per issued VALU instruction
  attainable  = frac / (issue_util x lane_util): the fraction the SAME
                instruction stream would reach at full issue with every
                instruction on 64 active lanes (the lane-ops packed into full
                waves). 1 / attainable is what the instruction stream itself
                costs against the op model; 1 / lane_util and 1 / issue_util
                are what divergence and stalls cost on top.

Per phase (a tools/phase_profile.py record), the wave-cycles each phase would
save at 64 lanes (its lanes per execution / 64) show where divergence costs.

    python tools/attainable.py --mix profiles/pmc_mix_c2.json --bench profiles/r6*_bench_c2.log
           [--phase profiles/r6*_phase_c2.json]
"""
import argparse
import json


def last_json(path):
    for line in reversed(open(path).read().splitlines()):
        line = line.strip()
        if line.startswith("{"):
            return json.loads(line)
    raise SystemExit(f"no JSON line in {path}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mix", required=True)
    ap.add_argument("--bench", required=True, help="a bench.py log (its last JSON line) of the same build")
    ap.add_argument("--phase", default=None)
    a = ap.parse_args()
    mix = json.load(open(a.mix))
    roof = last_json(a.bench)["roofline"]
    c = mix["counters"]
    fp64 = sum(c.get(k, 0.0) for k in ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64",
                                        "SQ_INSTS_VALU_TRANS_F64"))
    valu = c["SQ_INSTS_VALU"]
    issue_cycles = 4 * fp64 + 2 * (valu - fp64)
    simd_cycles = 1024 * c["GRBM_GUI_ACTIVE"] / 8
    issue_util = issue_cycles / simd_cycles
    lane_util = c["SQ_THREAD_CYCLES_VALU"] / (64 * c["SQ_ACTIVE_INST_VALU"])
    frac = roof["frac"]
    attainable = frac / (issue_util * lane_util)
    ops = roof["fp64_ops_per_launch"] + 0.5 * roof["fp32_ops_per_launch"]
    # executed lane-operations in FP64-op equivalents (an FP64 op = 1, any other VALU op = 1/2, as the model)
    lane_ops = (fp64 + 0.5 * (valu - fp64)) * 64 * lane_util
    out = {
        "frac": frac,
        "issue_util": round(issue_util, 4),
        "lane_util": round(lane_util, 4),
        "attainable_frac": round(attainable, 4),
        "cost_factors": {
            "instruction_stream_vs_op_model": round(1 / attainable, 3),
            "divergence": round(1 / lane_util, 3),
            "issue_stalls": round(1 / issue_util, 3),
        },
        "executed_lane_ops_over_model_ops": round(lane_ops / ops, 3),
        "fp64_share_of_valu": round(fp64 / valu, 4),
        "source": {"mix": a.mix, "bench": a.bench},
        "reading": "the same instructions at full issue on 64 active lanes would run at attainable_frac of the FP64 "
                   "roof; the rest of the gap is the instruction stream the parity contract and the algorithm "
                   "need per op of the model (CR sqrt/div, Philox, FP32 slab tests, compares/selects/moves)",
    }
    if a.phase:
        ph = last_json(a.phase)
        total = sum(ph[k] for k in ("cyc_refill", "cyc_node", "cyc_leaf", "cyc_shade"))
        lanes = {"cyc_refill": ph["lanes_per_refill_phase"], "cyc_node": ph["lanes_per_node_iter"],
                 "cyc_leaf": ph["lanes_per_leaf_phase"], "cyc_shade": ph["lanes_per_shade_phase"]}
        out["divergence_by_phase"] = {
            k[4:]: {"share": round(ph[k] / total, 3), "lanes": lanes[k],
                    "saved_at_64_lanes_share_of_frame": round(ph[k] * (1 - lanes[k] / 64) / total, 3)}
            for k in lanes}
        out["source"]["phase"] = a.phase
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
