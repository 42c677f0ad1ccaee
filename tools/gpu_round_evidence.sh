#!/bin/bash
# Round-end evidence for the committed tree (run on the GPU box from the repo
# root), in two parts that each fit one gpurun call:
#   part 1: smoke, GPU tests, the default bench line (C2), rocprof kernel-trace +
#           PMC + instruction mix of the bench shape, the N > 1 code path rehearsed
#           with gloo ranks on one GPU (parity of the gathered frame), and the
#           one-GPU rehearsal of the multi-GPU split (tools/shard_sim.py);
#   part 2: other configs' bench lines and their counter profiles (default c1 c3 c5).
#   usage: tools/gpu_round_evidence.sh <outdir> [1|2 [configs...]]
#   then:  python tools/pmc_summary.py <outdir>/prof/C/bench --config C --tag rN_C_f16 --frames 16
#          python tools/pmc_mix.py <outdir>/prof/C --config C --frames 16 > profiles/pmc_mix_C.json
set -u
O=${1:-gpurun_out/ev}; PART=${2:-1}; shift 2 2>/dev/null; CFGS=${*:-c1 c3 c5}; mkdir -p $O
if [ "$PART" = 1 ]; then
  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
  # A failing GPU suite ends the evidence run: no bench or profile may come from a red tree.
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 180 --timeout-method thread > $O/pytest.log 2>&1
  rc=$?; if [ $rc -ne 0 ]; then echo "pytest rc=$rc" > $O/FAILED; exit $rc; fi
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench_c2.log 2>&1 || exit 1
  O=$O/prof bash tools/profile_configs.sh c2 || exit 1
  for n in 2 4; do
    TRAY_BENCH_BACKEND=gloo timeout -k 10 300 python3 bench.py --gpus $n --steps 20 --warmup 5 > $O/bench_gloo$n.log 2>&1 || exit 1
  done
  timeout -k 10 300 python3 tools/shard_sim.py --ns 1,2,4,8 --passes 16 --frames-in-flight 2 --reps 24 > $O/shard_c2.jsonl 2>&1 || exit 1
else
  for c in $CFGS; do
    timeout -k 10 400 python3 bench.py --config $c --steps 20 --warmup 5 > $O/bench_$c.log 2>&1 || exit 1
  done
  O=$O/prof bash tools/profile_configs.sh $CFGS || exit 1
fi
echo ok > $O/done$PART
