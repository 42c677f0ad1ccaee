#!/bin/bash
# Round-end evidence for the committed tree (run on the GPU box from the repo
# root): GPU tests, the default bench line, rocprof stats/PMC, other configs,
# and the one-GPU multi-GPU rehearsal (tools/shard_sim.py).
#   usage: tools/gpu_round_evidence.sh <outdir>
set -u
O=${1:-gpurun_out/ev}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py > $O/bench_c2.log 2>&1 || exit 1
bash tools/gpu_profile_all.sh $O/all || exit 1
for c in c1 c3 c5; do
  timeout -k 10 300 python3 bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_$c.log 2>&1 || exit 1
done
timeout -k 10 300 python3 tools/shard_sim.py --ns 1,2,4,8 --passes 8 --frames-in-flight 2 --reps 24 > $O/shard_p8.jsonl 2>&1 || exit 1
echo ok > $O/done
