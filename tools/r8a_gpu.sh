set -u
O=gpurun_out/r8a; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench_c2.json 2> $O/bench_c2.err || exit 1
timeout -k 10 300 python3 bench.py --config c1 --steps 20 --warmup 5 > $O/bench_c1.json 2> $O/bench_c1.err || exit 1
echo done
