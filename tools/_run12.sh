set -o pipefail
O=gpurun_out/adapt; mkdir -p $O
V=tray_amd/build/variants
A="base=tray_amd/libtray_amd.so"
for v in a6m40 a6m32 a2x6m32 a5m48 lb16 lb20; do A="$A $v=$V/$v/libtray_amd.so"; done
timeout -k 10 400 python3 tools/ab_bench.py --config c2 --rounds 7 $A > $O/ab_c2.jsonl 2>&1 || exit 1
timeout -k 10 400 python3 tools/ab_bench.py --config c5 --rounds 2 $A > $O/ab_c5.jsonl 2>&1 || exit 1
echo ok > $O/done
