#!/bin/bash
# Latency counters of the C2 megakernel (16-frame launches): LDS, instruction fetch, VMEM, SMEM
# (rocprofv3 derived metrics: accumulated in-flight level / instruction count), one pass each pair.
set -u
O=gpurun_out/lat; mkdir -p $O
export TMPDIR=/tmp
ARGS="--steps 16 --warmup 0 --no-cpu-baseline --no-e2e --no-single --frames-in-flight 1"
i=0
for SET in "LdsLatency InstrFetchLatency" "VmemLatency SmemLatency" \
           "SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_SALU SQ_INSTS_LDS_LOAD SQ_INSTS_LDS_STORE SQ_INSTS_LDS_ATOMIC SQ_INSTS_VSKIPPED"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $SET --kernel-include-regex render_kernel -d "$O/p$i" -o pmc \
      --output-format csv -- python3 bench.py $ARGS > "$O/p$i.log" 2>&1
  rc=$?; echo "pass $i ($SET) rc=$rc" | tee -a "$O/status.txt"
  [ $rc -eq 0 ] || exit $rc
done
