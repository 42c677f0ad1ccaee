set -o pipefail
O=gpurun_out/r2c_check; mkdir -p $O
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench_c2.log 2>&1 || exit 1
echo ok > $O/done
