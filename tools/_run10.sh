set -o pipefail
O=gpurun_out/gskip; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_candidates.py tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
timeout -k 10 300 python3 tools/ab_bench.py --config c2 --rounds 6 head=tray_amd/build/variants/head/libtray_amd.so gskip=tray_amd/libtray_amd.so > $O/ab_c2.jsonl 2>&1 || exit 1
timeout -k 10 300 python3 tools/ab_bench.py --config c5 --rounds 2 head=tray_amd/build/variants/head/libtray_amd.so gskip=tray_amd/libtray_amd.so > $O/ab_c5.jsonl 2>&1 || exit 1
echo ok > $O/done
