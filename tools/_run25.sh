set -o pipefail
O=gpurun_out/f16; mkdir -p $O
V=tray_amd/build/variants
B="--steps 32 --warmup 4 --no-cpu-baseline --no-e2e --no-single"
for rep in 1 2; do
  timeout -k 10 150 python3 bench.py $B --passes 8 > $O/f8_$rep.log 2>&1 || exit 1
  TRAY_LIB=$V/b30/libtray_amd.so timeout -k 10 150 python3 bench.py $B --passes 16 > $O/f16_$rep.log 2>&1 || exit 1
done
timeout -k 10 300 python3 tools/shard_sim.py --ns 1,8 --passes 8 --frames-in-flight 2 --reps 16 > $O/shard_f8.jsonl 2>&1 || exit 1
timeout -k 10 300 python3 tools/shard_sim.py --ns 1,8 --passes 16 --frames-in-flight 2 --reps 16 --lib $V/b30/libtray_amd.so > $O/shard_f16.jsonl 2>&1 || exit 1
timeout -k 10 150 python3 bench.py --config c1 $B --passes 8 > $O/c1_f8.log 2>&1 || exit 1
TRAY_LIB=$V/b30/libtray_amd.so timeout -k 10 150 python3 bench.py --config c1 $B --passes 16 > $O/c1_f16.log 2>&1 || exit 1
echo ok > $O/done
