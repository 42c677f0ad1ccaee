set -o pipefail
O=gpurun_out/cand3; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_candidates.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python3 bench.py --steps 8 --warmup 0 --no-cpu-baseline --no-single --frames-in-flight 1 > $O/kt.log 2>&1 || exit 1
for c in c3 c5; do timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_$c -o kt --output-format csv -- python3 bench.py --config $c --steps 2 --warmup 0 --no-cpu-baseline --no-single --frames-in-flight 1 > $O/kt_$c.log 2>&1 || exit 1; done
bash tools/_run12.sh || exit 1
echo ok > $O/done
