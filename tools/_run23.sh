set -o pipefail
O=gpurun_out/cores2; mkdir -p $O
V=tray_amd/build/variants
B="--steps 24 --warmup 4 --no-cpu-baseline --no-e2e --no-single"
for rep in 1 2; do
  timeout -k 10 120 python3 bench.py $B > $O/base_$rep.log 2>&1 || exit 1
  TRAY_LIB=$V/v120nt/libtray_amd.so TRAY_RESOLVE_LEAN=1 timeout -k 10 120 python3 bench.py $B > $O/v120nt_$rep.log 2>&1 || exit 1
  TRAY_LIB=$V/v120/libtray_amd.so TRAY_RESOLVE_LEAN=1 timeout -k 10 120 python3 bench.py $B > $O/v120lean_$rep.log 2>&1 || exit 1
done
echo ok > $O/done
