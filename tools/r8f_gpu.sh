#!/bin/bash
# Round 5 evidence for the committed tree (tools/gpu_round_evidence.sh plus the
# e2e split): smoke, GPU suite, bench lines with parity and CPU baselines,
# kernel trace + HBM/instruction-mix counters + phase split, shard rehearsal.
set -u
O=gpurun_out/r8f
bash tools/gpu_round_evidence.sh $O || exit 1
timeout -k 10 120 python3 tools/e2e_split.py --config c2 > $O/e2e_split.json 2> $O/e2e_split.err || exit 1
echo ok > $O/all_done
