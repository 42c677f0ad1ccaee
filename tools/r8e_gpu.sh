#!/bin/bash
# Round 5: guided chunk reservations (the reservation shrinks with the chunks left,
# instead of 32-chunk reservations and single-chunk takes for the last 8
# reservations' worth) at N = 1 (A/B) and in the one-GPU rehearsal of the 8-way split.
set -u
O=gpurun_out/r8e; mkdir -p $O
V=tray_amd/build/variants
timeout -k 10 400 python3 tools/ab_bench.py --config c2 --passes 16 --rounds 7 base=$V/base/libtray_amd.so gbase=$V/gbase/libtray_amd.so g1=$V/g1/libtray_amd.so g2=$V/g2/libtray_amd.so g3=$V/g3/libtray_amd.so > $O/ab_c2.jsonl 2>&1 || exit 1
timeout -k 10 400 python3 tools/ab_bench.py --config c5 --passes 16 --rounds 3 base=$V/base/libtray_amd.so g1=$V/g1/libtray_amd.so g2=$V/g2/libtray_amd.so g3=$V/g3/libtray_amd.so > $O/ab_c5.jsonl 2>&1 || exit 1
for v in base g1 g2 g3; do
  timeout -k 10 300 python3 tools/shard_sim.py --lib $V/$v/libtray_amd.so --ns 1,8 --passes 16 --frames-in-flight 2 --reps 24 > $O/shard_$v.jsonl 2>&1 || exit 1
done
echo done > $O/done
