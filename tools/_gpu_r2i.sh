# round-2 evidence for the current tree: smoke, GPU tests, bench line, kernel-trace + PMC + phase profiles
O=gpurun_out/r2i; mkdir -p $O
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc" > $O/status
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 180 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/status
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1; echo "bench rc=$?" >> $O/status
bash tools/gpu_profile_all.sh $O/all; echo "profile rc=$?" >> $O/status
