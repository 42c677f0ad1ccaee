# round-2: GPU tests (progress instance), bench line, one-GPU rehearsal of the 8-way split in the bench shape
O=gpurun_out/r2e; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 180 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" > $O/status
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1; echo "bench rc=$?" >> $O/status
timeout -k 10 300 python3 tools/shard_sim.py --ns 1,2,4,8 --passes 8 --frames-in-flight 2 --reps 24 > $O/shard_c2.jsonl 2>$O/shard_c2.err; echo "shard rc=$?" >> $O/status
for c in c3 c5; do timeout -k 10 300 python3 bench.py --config $c --steps 8 --warmup 1 --no-cpu-baseline > $O/bench_$c.log 2>&1; echo "bench $c rc=$?" >> $O/status; done
