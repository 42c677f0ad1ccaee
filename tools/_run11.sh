set -o pipefail
O=gpurun_out/cand2; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_candidates.py -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
echo ok > $O/done
