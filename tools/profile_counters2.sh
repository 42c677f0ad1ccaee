#!/bin/bash
# Second set of counter passes for the render kernel (issue mix, LDS, fetch).
#   usage: tools/profile_counters2.sh <outdir> [bench.py args...]
set -u
OUT=${1:-gpurun_out/pmc2}; shift || true
ARGS=${*:-"--steps 16 --warmup 0 --no-cpu-baseline --no-e2e --no-single --frames-in-flight 1"}
export TMPDIR=/tmp
mkdir -p "$OUT"
# the device code these counters describe (bench.py only reuses them for the same code)
python3 -c "from tray_amd import _lib; print(_lib.code_object_sha256())" > "$OUT/code_object_sha256.txt" || exit 1
i=0
for SET in \
  "SQ_ACTIVE_INST_VALU2 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_TRANS_F32 SQ_WAIT_INST_LDS SQ_INSTS_LDS" \
  "SQ_IFETCH SQ_INSTS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_LEVEL_LDS SQ_LDS_ADDR_CONFLICT SQ_CYCLES" ; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $SET --kernel-include-regex render_kernel -d "$OUT/p$i" -o pmc \
      --output-format csv -- python3 bench.py $ARGS > "$OUT/p$i.log" 2>&1
  echo "pass $i rc=$?" >> "$OUT/status.txt"
done
