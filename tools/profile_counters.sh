#!/bin/bash
# Counter passes for the render kernel (run on the GPU box from the repo root).
# Each --pmc pass is its own rocprofv3 run (never combined with tracing domains).
#   usage: tools/profile_counters.sh <outdir> [bench.py args...]
set -u
OUT=${1:-gpurun_out/pmc}; shift || true
ARGS=${*:-"--steps 16 --warmup 0 --no-cpu-baseline --no-e2e --no-single --frames-in-flight 1"}
export TMPDIR=/tmp
mkdir -p "$OUT"
# the device code these counters describe (bench.py only reuses them for the same code)
python3 -c "from tray_amd import _lib; print(_lib.code_object_sha256())" > "$OUT/code_object_sha256.txt" || exit 1
i=0
for SET in \
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU" \
  "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_INT32" \
  "GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU_INT64 SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_VALU_FLOPS_FP64" ; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $SET --kernel-include-regex render_kernel -d "$OUT/p$i" -o pmc \
      --output-format csv -- python3 bench.py $ARGS > "$OUT/p$i.log" 2>&1
  echo "pass $i rc=$?" >> "$OUT/status.txt"
done
