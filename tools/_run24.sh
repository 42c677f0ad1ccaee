set -o pipefail
O=gpurun_out/ntst; mkdir -p $O
V=tray_amd/build/variants
B="--steps 24 --warmup 4 --no-cpu-baseline --no-e2e --no-single"
timeout -k 10 300 python3 tools/ab_bench.py --config c2 --rounds 6 base=tray_amd/libtray_amd.so ntst=$V/ntst/libtray_amd.so > $O/ab_c2.jsonl 2>&1 || exit 1
timeout -k 10 300 python3 tools/ab_bench.py --config c5 --rounds 2 base=tray_amd/libtray_amd.so ntst=$V/ntst/libtray_amd.so > $O/ab_c5.jsonl 2>&1 || exit 1
for rep in 1 2; do
  timeout -k 10 120 python3 bench.py $B > $O/base_$rep.log 2>&1 || exit 1
  TRAY_LIB=$V/ntst/libtray_amd.so timeout -k 10 120 python3 bench.py $B > $O/ntst_$rep.log 2>&1 || exit 1
done
echo ok > $O/done
