#!/bin/bash
# Lane utilisation of an N-way shard (A) against the whole frame (B) over the same
# samples, for several splits: which property of the split costs (tools/shard_pmc.py).
#   usage: tools/shard_pmc2.sh <outdir>
set -u
OUT=${1:-gpurun_out/shard_pmc2}
export TMPDIR=/tmp
mkdir -p "$OUT"
C="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS"
for CASE in "8 1 16" "8 8 16" "9 1 18" "2 1 16" "4 1 16"; do
  set -- $CASE
  D="$OUT/n$1_t$2"
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex render_kernel -d "$D" -o pmc --output-format csv \
      -- python3 tools/shard_pmc.py --n $1 --tile-rows $2 --passes $3 --reps 4 > "$D.log" 2>&1 || exit 1
  python3 tools/shard_pmc.py --summarize "$D" > "$D.json" || exit 1
done
echo ok > "$OUT/done"
