#!/bin/bash
set -u
O=gpurun_out/e7; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
timeout -k 10 300 python3 tools/ab_bench.py --rounds 9 bu=tray_amd/build/variants/bu/libtray_amd.so td=tray_amd/build/variants/td/libtray_amd.so > $O/ab.jsonl 2>&1 || exit 1
for L in bu td; do
  timeout -k 10 300 python3 tools/shard_sim.py --ns 1,2,4,8 --frames-in-flight 3 --reps 24 --lib tray_amd/build/variants/$L/libtray_amd.so > $O/shard_${L}_f3.jsonl 2>&1 || exit 1
done
timeout -k 10 300 python3 tools/shard_sim.py --ns 1,8 --frames-in-flight 1 --reps 9 --lib tray_amd/build/variants/bu/libtray_amd.so > $O/shard_bu_f1.jsonl 2>&1 || exit 1
