#!/bin/bash
# One GPU call's worth of evidence for the current tree (run on the GPU box from
# the repo root): kernel-trace stats + HBM counters of the bench command, the
# instruction-mix counter passes, and the -DTRAY_PROFILE phase split.
#   usage: tools/gpu_profile_all.sh <outdir> [config]
set -u
OUT=${1:-gpurun_out/all}
CFG=${2:-c2}
mkdir -p "$OUT"
A="--config $CFG --steps 16 --warmup 0 --no-cpu-baseline --no-e2e --no-single --frames-in-flight 1"
bash tools/profile_bench.sh "$OUT/bench" $A || exit 1
bash tools/profile_counters.sh "$OUT/pmc1" $A || exit 1
bash tools/profile_counters2.sh "$OUT/pmc2" $A || exit 1
if [ -f tray_amd/build/variants/prof/libtray_amd.so ]; then
  timeout -k 10 120 python3 tools/phase_profile.py tray_amd/build/variants/prof/libtray_amd.so --config $CFG > "$OUT/phase.json" 2>"$OUT/phase.err" || exit 1
fi
echo ok > "$OUT/done"
