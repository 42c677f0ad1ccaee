# round-2 GPU check: progress/C-caller tests, then kernel-trace + PMC + phase profiles of the bench shape
O=gpurun_out/r2b; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_tracer.py tests/test_c_caller.py -m gpu -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" > $O/status
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/gpu_profile_all.sh $O/all; echo "profile rc=$?" >> $O/status
