#!/bin/bash
# C1 (the reference's benchmark/ config): on-chip pixel-pass sums (grp) against the FP64
# sample-order sum (ord, the previous default for r = 16), longer interleaved runs.
set -u
O=gpurun_out/r9d; mkdir -p $O
L=tray_amd/libtray_amd.so
for P in 16 1; do
  R=$([ $P = 1 ] && echo 61 || echo 25)
  timeout -k 10 300 python -u tools/ab_bench.py --config c1 --rounds $R --passes $P \
      grp=$L ord=$L@ordered_sum=1 > $O/ab_c1_p$P.jsonl 2>&1 || { tail -20 $O/ab_c1_p$P.jsonl; exit 1; }
  grep variant $O/ab_c1_p$P.jsonl
done
timeout -k 10 300 python -u bench.py --config c1 --no-cpu-baseline > $O/bench_c1.log 2>&1 || { tail -20 $O/bench_c1.log; exit 1; }
tail -1 $O/bench_c1.log | cut -c1-400
