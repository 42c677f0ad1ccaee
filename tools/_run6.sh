set -o pipefail
O=gpurun_out/cand1; mkdir -p $O
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_candidates.py -x -v --timeout 120 --timeout-method thread > $O/pytest_cand.log 2>&1 || exit 1
timeout -k 10 240 python3 tools/ab_bench.py --config c2 --rounds 5 nocand=tray_amd/libtray_amd.so@TRAY_PRIMARY_CANDIDATES=0 cand=tray_amd/libtray_amd.so@TRAY_PRIMARY_CANDIDATES=1 > $O/ab_c2.jsonl 2>&1 || exit 1
timeout -k 10 240 python3 tools/ab_bench.py --config c5 --rounds 3 nocand=tray_amd/libtray_amd.so@TRAY_PRIMARY_CANDIDATES=0 cand=tray_amd/libtray_amd.so@TRAY_PRIMARY_CANDIDATES=1 > $O/ab_c5.jsonl 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > $O/pytest_all.log 2>&1 || exit 1
echo ok > $O/done
