#!/bin/bash
set -u
O=gpurun_out/r8j; mkdir -p $O
TRAY_BENCH_BACKEND=gloo timeout -k 10 300 python3 bench.py --gpus 2 --steps 20 --warmup 5 > $O/gloo2.json 2> $O/gloo2.err || exit 1
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_c2.json 2> $O/bench_c2.err || exit 1
echo done > $O/done
