#!/bin/bash
# bench.py with one device scene shared by its frame slots: the bench-path test,
# the default line and the N = 2 gloo rehearsal.
set -u
O=gpurun_out/r8h; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_bench_path.py tests/test_gpu_scene_concurrency.py -m gpu -x -v --timeout 180 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench_c2.json 2> $O/bench_c2.err || exit 1
TRAY_BENCH_BACKEND=gloo timeout -k 10 300 python3 bench.py --gpus 2 --steps 20 --warmup 5 > $O/gloo2.json 2> $O/gloo2.err || exit 1
echo done > $O/done
