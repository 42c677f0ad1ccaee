set -o pipefail
O=gpurun_out/sparse3; mkdir -p $O
V=tray_amd/build/variants
A="head=$V/head/libtray_amd.so cur=tray_amd/libtray_amd.so"
for v in rl8 rl12 rl16 nss1 nss2 rl12nss1; do A="$A $v=$V/$v/libtray_amd.so"; done
timeout -k 10 500 python3 tools/ab_bench.py --config c2 --rounds 7 $A > $O/ab_c2.jsonl 2>&1 || exit 1
timeout -k 10 500 python3 tools/ab_bench.py --config c5 --rounds 2 $A > $O/ab_c5.jsonl 2>&1 || exit 1
echo ok > $O/done
