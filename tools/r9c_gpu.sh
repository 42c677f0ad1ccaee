#!/bin/bash
# On-chip sums for r = 16 / 32 (one record per pixel-pass): accumulation and parity tests,
# then C1 timed against the FP64 sample-order sum and the per-sample buffer (same library).
set -u
O=gpurun_out/r9c; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_accum.py tests/test_gpu_parity.py tests/test_gpu_bench_path.py \
    -x -v --timeout 180 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
L=tray_amd/libtray_amd.so
for P in 16 1; do
  timeout -k 10 300 python -u tools/ab_bench.py --config c1 --rounds 15 --passes $P \
      grp=$L ord=$L@ordered_sum=1 buf=$L@acc_slots=0 > $O/ab_c1_p$P.jsonl 2>&1 || { tail -20 $O/ab_c1_p$P.jsonl; exit 1; }
  cat $O/ab_c1_p$P.jsonl
done
