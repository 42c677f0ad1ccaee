set -o pipefail
O=gpurun_out/sf; mkdir -p $O
V=tray_amd/build/variants
A="base=tray_amd/libtray_amd.so"
for v in sf1 sf2 sf1sb32 sf1sb48 sf2sb48; do A="$A $v=$V/$v/libtray_amd.so"; done
timeout -k 10 400 python3 tools/ab_bench.py --config c2 --rounds 6 $A > $O/ab_c2.jsonl 2>&1 || exit 1
timeout -k 10 400 python3 tools/ab_bench.py --config c5 --rounds 2 $A > $O/ab_c5.jsonl 2>&1 || exit 1
echo ok > $O/done
