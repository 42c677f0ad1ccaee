set -o pipefail
O=gpurun_out/sparse2; mkdir -p $O
V=tray_amd/build/variants
A="head=$V/head/libtray_amd.so ts8s16l8=$V/ts8s16l8/libtray_amd.so"
for v in ts8l8 ts12s16l8 ts8s12l6 ts8s20l8 ts4s16l4; do A="$A $v=$V/$v/libtray_amd.so"; done
timeout -k 10 500 python3 tools/ab_bench.py --config c2 --rounds 7 $A > $O/ab_c2.jsonl 2>&1 || exit 1
timeout -k 10 500 python3 tools/ab_bench.py --config c5 --rounds 2 $A > $O/ab_c5.jsonl 2>&1 || exit 1
echo ok > $O/done
