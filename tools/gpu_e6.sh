#!/bin/bash
set -u
O=gpurun_out/e6; mkdir -p $O
timeout -k 10 300 python3 tools/ab_bench.py --rounds 9 main=tray_amd/build/variants/main/libtray_amd.so b512=tray_amd/build/variants/b512/libtray_amd.so b256=tray_amd/build/variants/b256/libtray_amd.so lb12=tray_amd/build/variants/lb12/libtray_amd.so lb16=tray_amd/build/variants/lb16/libtray_amd.so lb20=tray_amd/build/variants/lb20/libtray_amd.so > $O/ab.jsonl 2>&1 || exit 1
for f in 3 6; do
  timeout -k 10 300 python3 tools/shard_sim.py --ns 1,8 --frames-in-flight $f --reps 24 --lib tray_amd/build/variants/main/libtray_amd.so > $O/shard_main_f$f.jsonl 2>&1 || exit 1
  timeout -k 10 300 python3 tools/shard_sim.py --ns 1,8 --frames-in-flight $f --reps 24 --lib tray_amd/build/variants/b512/libtray_amd.so > $O/shard_b512_f$f.jsonl 2>&1 || exit 1
done
