#!/bin/bash
set -u
O=gpurun_out/e10; mkdir -p $O
export MASTER_ADDR=127.0.0.1
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
timeout -k 10 200 python3 bench.py > $O/bench.log 2>&1 || exit 1
timeout -k 10 200 python3 bench.py --passes 8 --steps 16 --no-cpu-baseline > $O/bench_p8.log 2>&1 || exit 1
TRAY_BENCH_BACKEND=gloo timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29555 bench.py --gpus 2 --steps 16 --warmup 8 > $O/bench_gloo2.log 2>&1 || exit 1
TRAY_BENCH_BACKEND=gloo timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29556 bench.py --gpus 4 --steps 10 --warmup 2 --passes 3 > $O/bench_gloo4.log 2>&1 || exit 1
