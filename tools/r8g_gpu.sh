#!/bin/bash
# Round 5: branch-free node step (bf), branch-free leaf pop (lbf), both (bfl) against the product kernel.
set -u
O=gpurun_out/r8g; mkdir -p $O
V=tray_amd/build/variants
timeout -k 10 400 python3 tools/ab_bench.py --config c2 --passes 16 --rounds 9 base=$V/base/libtray_amd.so bf=$V/bf/libtray_amd.so lbf=$V/lbf/libtray_amd.so bfl=$V/bfl/libtray_amd.so > $O/ab_c2.jsonl 2>&1 || exit 1
timeout -k 10 400 python3 tools/ab_bench.py --config c5 --passes 16 --rounds 4 base=$V/base/libtray_amd.so bf=$V/bf/libtray_amd.so lbf=$V/lbf/libtray_amd.so bfl=$V/bfl/libtray_amd.so > $O/ab_c5.jsonl 2>&1 || exit 1
timeout -k 10 300 python3 tools/ab_bench.py --config c1 --passes 16 --rounds 9 base=$V/base/libtray_amd.so bf=$V/bf/libtray_amd.so bfl=$V/bfl/libtray_amd.so > $O/ab_c1.jsonl 2>&1 || exit 1
echo done > $O/done
