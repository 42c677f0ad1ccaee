set -o pipefail
O=gpurun_out/cores; mkdir -p $O
V=tray_amd/build/variants
B="--steps 24 --warmup 4 --no-cpu-baseline --no-e2e --no-single"
for rep in 1 2; do
  timeout -k 10 120 python3 bench.py $B > $O/base_$rep.log 2>&1 || exit 1
  TRAY_RESOLVE_LEAN=1 timeout -k 10 120 python3 bench.py $B > $O/lean_$rep.log 2>&1 || exit 1
  TRAY_LIB=$V/v120/libtray_amd.so timeout -k 10 120 python3 bench.py $B > $O/v120_$rep.log 2>&1 || exit 1
  TRAY_LIB=$V/v120/libtray_amd.so TRAY_RESOLVE_LEAN=1 timeout -k 10 120 python3 bench.py $B > $O/v120lean_$rep.log 2>&1 || exit 1
done
timeout -k 10 300 python3 tools/ab_bench.py --config c2 --rounds 5 base=tray_amd/libtray_amd.so v120=$V/v120/libtray_amd.so > $O/ab_c2.jsonl 2>&1 || exit 1
echo ok > $O/done
