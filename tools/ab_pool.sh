#!/bin/bash
# A/B of the workgroup pool size (TRAY_POOL_CHUNKS) on the round-4 work order.
#   tools/build_variants.sh base "" p128 "-DTRAY_POOL_CHUNKS=128" p256 "-DTRAY_POOL_CHUNKS=256" p32 "-DTRAY_POOL_CHUNKS=32"
set -u
O=${1:-gpurun_out/pool}; mkdir -p $O
V=""; for v in base p128 p256 p32; do V="$V $v=tray_amd/build/variants/$v/libtray_amd.so"; done
timeout -k 10 300 python3 tools/ab_bench.py --config c2 --passes 16 --rounds 8 $V > $O/ab_c2_f16.jsonl 2>$O/err1 || exit 1
timeout -k 10 300 python3 tools/ab_bench.py --config c5 --passes 16 --rounds 2 $V > $O/ab_c5_f16.jsonl 2>$O/err2 || exit 1
for v in base p128 p256 p32; do
  timeout -k 10 300 python3 tools/shard_sim.py --ns 8 --passes 16 --frames-in-flight 2 --reps 24 --lib tray_amd/build/variants/$v/libtray_amd.so > $O/shard_$v.jsonl 2>$O/err_$v || exit 1
done
echo ok > $O/done
