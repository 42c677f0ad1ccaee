set -o pipefail
O=gpurun_out/spec3; mkdir -p $O
TRAY_SPEC=1 TRAY_LIB=tray_amd/build/variants/specwd/libtray_amd.so timeout -k 10 60 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 180 python3 tools/ab_bench.py --config c2 --rounds 5 base=tray_amd/libtray_amd.so spec=tray_amd/build/variants/specwd/libtray_amd.so@TRAY_SPEC=1 > $O/ab_c2.jsonl 2>&1 || exit 1
timeout -k 10 180 python3 tools/ab_bench.py --config c5 --rounds 3 base=tray_amd/libtray_amd.so spec=tray_amd/build/variants/specwd/libtray_amd.so@TRAY_SPEC=1 > $O/ab_c5.jsonl 2>&1 || exit 1
TRAY_SPEC=1 TRAY_LIB=tray_amd/build/variants/specwd/libtray_amd.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
echo ok > $O/done
