#!/bin/bash
# Round 5: accumulator runs (one chunk record per run of up to 4 chunks at r >= 128):
# the GPU suite on the new build, A/B against the round-4 kernel (base), and the
# C3 HBM counters of the new build.
set -u
O=gpurun_out/r8d; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; if [ $rc -ne 0 ]; then exit $rc; fi
V=tray_amd/build/variants
timeout -k 10 300 python3 tools/ab_bench.py --config c2 --passes 16 --rounds 7 base=$V/base/libtray_amd.so runs=$V/runs/libtray_amd.so > $O/ab_c2.jsonl 2>&1 || exit 1
timeout -k 10 600 python3 tools/ab_bench.py --config c3 --passes 16 --rounds 3 base=$V/base/libtray_amd.so runs=$V/runs/libtray_amd.so > $O/ab_c3.jsonl 2>&1 || exit 1
timeout -k 10 300 python3 tools/ab_bench.py --config c5 --passes 16 --rounds 5 base=$V/base/libtray_amd.so runs=$V/runs/libtray_amd.so > $O/ab_c5.jsonl 2>&1 || exit 1
bash tools/profile_bench.sh $O/prof_c3 --config c3 --steps 16 --warmup 0 --no-cpu-baseline --no-e2e --no-single --frames-in-flight 1 || exit 1
echo done > $O/done
