#!/bin/bash
# Round 5, first GPU call: the GPU suite, the C2 and C1 bench lines, and the
# LDS-layout A/B (axis-pair node layout vs 128-B nodes, and the no-add probe).
set -u
O=gpurun_out/r8b; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench_c2.json 2> $O/bench_c2.err || exit 1
timeout -k 10 300 python3 bench.py --config c1 --steps 20 --warmup 5 > $O/bench_c1.json 2> $O/bench_c1.err || exit 1
V=tray_amd/build/variants
timeout -k 10 300 python3 tools/ab_bench.py --config c2 --passes 16 --rounds 9 base=$V/base/libtray_amd.so pairs=$V/pairs/libtray_amd.so noadd=$V/noadd/libtray_amd.so > $O/ab_c2.jsonl 2>&1 || exit 1
timeout -k 10 300 python3 tools/ab_bench.py --config c5 --passes 16 --rounds 5 base=$V/base/libtray_amd.so pairs=$V/pairs/libtray_amd.so > $O/ab_c5.jsonl 2>&1 || exit 1
A="--steps 16 --warmup 0 --no-cpu-baseline --no-e2e --no-single --frames-in-flight 1"
for v in base pairs noadd; do
  TRAY_LIB=$V/$v/libtray_amd.so timeout -k 10 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU --kernel-include-regex render_kernel -d $O/pmc_$v -o pmc --output-format csv -- python3 bench.py $A > $O/pmc_$v.log 2>&1 || exit 1
done
timeout -k 10 120 python3 tools/e2e_split.py --config c2 > $O/e2e_split.json 2>$O/e2e_split.err || exit 1
echo done > $O/done
