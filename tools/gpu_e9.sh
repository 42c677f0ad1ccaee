#!/bin/bash
set -u
O=gpurun_out/e9; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
for cfg in "1 3" "2 2" "4 2" "8 2" "4 1" "2 1"; do
  set -- $cfg
  timeout -k 10 300 python3 tools/shard_sim.py --ns 1,8 --passes $1 --frames-in-flight $2 --reps 24 > $O/shard_p$1_f$2.jsonl 2>&1 || exit 1
done
