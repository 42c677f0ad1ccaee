#!/bin/bash
# Counter passes of tools/shard_pmc.py (run on the GPU box from the repo root).
#   usage: tools/shard_pmc.sh <outdir>
set -u
OUT=${1:-gpurun_out/shard_pmc}
export TMPDIR=/tmp
mkdir -p "$OUT"
timeout -k 10 120 python3 tools/shard_pmc.py --n 8 --reps 6 > "$OUT/times.json" 2>"$OUT/times.err" || exit 1
i=0
for SET in \
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU" \
  "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_INT32" \
  "GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU_INT64 SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_VALU_FLOPS_FP64" ; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $SET --kernel-include-regex render_kernel -d "$OUT/p$i" -o pmc \
      --output-format csv -- python3 tools/shard_pmc.py --n 8 --reps 6 > "$OUT/p$i.log" 2>&1 || exit 1
done
python3 tools/shard_pmc.py --summarize "$OUT"/p1 "$OUT"/p2 "$OUT"/p3 > "$OUT/summary.json" || exit 1
echo ok > "$OUT/done"
