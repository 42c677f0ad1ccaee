set -o pipefail
O=gpurun_out/sparse; mkdir -p $O
V=tray_amd/build/variants
A="head=$V/head/libtray_amd.so cur=tray_amd/libtray_amd.so"
for v in ts16s24 ts16s24l12 ts24s24 ts16s16 ts8s16l8; do A="$A $v=$V/$v/libtray_amd.so"; done
timeout -k 10 500 python3 tools/ab_bench.py --config c2 --rounds 6 $A > $O/ab_c2.jsonl 2>&1 || exit 1
timeout -k 10 500 python3 tools/ab_bench.py --config c5 --rounds 2 $A > $O/ab_c5.jsonl 2>&1 || exit 1
echo ok > $O/done
