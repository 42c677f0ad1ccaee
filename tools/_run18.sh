set -o pipefail
O=gpurun_out/rs2; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
V=tray_amd/build/variants
A="base=tray_amd/libtray_amd.so"
for v in sb32 sb36 sb44 lb20 lb28 ns2 ns4 rb20 rb28; do A="$A $v=$V/$v/libtray_amd.so"; done
timeout -k 10 500 python3 tools/ab_bench.py --config c2 --rounds 6 $A > $O/ab_c2.jsonl 2>&1 || exit 1
timeout -k 10 500 python3 tools/ab_bench.py --config c5 --rounds 2 $A > $O/ab_c5.jsonl 2>&1 || exit 1
echo ok > $O/done
