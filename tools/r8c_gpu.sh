#!/bin/bash
# Round 5: the N > 1 bench path rehearsed on one GPU (gloo ranks sharing device 0:
# code path and the per-rank fields only, numbers meaningless), and the other
# configs' bench lines with their parity records (sampled rows at C3/C4/C5).
set -u
O=gpurun_out/r8c; mkdir -p $O
for n in 2 4; do
  TRAY_BENCH_BACKEND=gloo timeout -k 10 400 python3 bench.py --gpus $n --steps 20 --warmup 5 > $O/gloo$n.json 2> $O/gloo$n.err || exit 1
done
for c in c3 c5 c4; do
  timeout -k 10 400 python3 bench.py --config $c --steps 20 --warmup 5 > $O/bench_$c.json 2> $O/bench_$c.err || exit 1
done
echo done > $O/done
