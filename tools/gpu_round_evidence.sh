#!/bin/bash
# Round-end evidence for the committed tree (run on the GPU box from the repo
# root): smoke, GPU tests, the default bench line, rocprof kernel-trace + PMC +
# phase profiles of the bench shape, the other configs, and the one-GPU
# rehearsal of the multi-GPU split in the bench shape (tools/shard_sim.py).
#   usage: tools/gpu_round_evidence.sh <outdir>
#   then:  python tools/pmc_summary.py <outdir>/all/bench --config c2 --tag rN_c2_f16 --frames 16
#          python tools/pmc_mix.py <outdir>/all --frames 16 > profiles/pmc_mix_c2.json
set -u
O=${1:-gpurun_out/ev}; mkdir -p $O
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
# A failing GPU suite ends the evidence run: no bench or profile may come from a red tree.
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 180 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; if [ $rc -ne 0 ]; then echo "pytest rc=$rc" > $O/FAILED; exit $rc; fi
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench_c2.log 2>&1 || exit 1
bash tools/gpu_profile_all.sh $O/all || exit 1
# the other configs in the headline launch shape (the driver's --steps 20 --warmup 5: 16-frame launches)
for c in c1 c3 c5; do
  timeout -k 10 400 python3 bench.py --config $c --steps 20 --warmup 5 > $O/bench_$c.log 2>&1 || exit 1
done
timeout -k 10 300 python3 tools/shard_sim.py --ns 1,2,4,8 --passes 16 --frames-in-flight 2 --reps 24 > $O/shard_c2.jsonl 2>&1 || exit 1
echo ok > $O/done
