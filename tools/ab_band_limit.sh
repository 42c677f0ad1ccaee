#!/bin/bash
# A/B of the launch-band limit with on-chip chunk sums: 2^31 samples (the build) against
# 2^30 (the band_samples knob, the limit before round 4's end), same library, interleaved.
set -u
O=${1:-gpurun_out/band}; mkdir -p $O
V="b31=tray_amd/libtray_amd.so b30=tray_amd/libtray_amd.so@band_samples=1073741824"
timeout -k 10 300 python3 tools/ab_bench.py --config c5 --passes 16 --rounds 4 $V > $O/ab_c5_f16.jsonl 2>$O/err1 || exit 1
timeout -k 10 300 python3 tools/ab_bench.py --config c3 --passes 16 --rounds 3 $V > $O/ab_c3_f16.jsonl 2>$O/err2 || exit 1
timeout -k 10 300 python3 tools/ab_bench.py --config c4 --passes 1 --rounds 3 $V > $O/ab_c4_f1.jsonl 2>$O/err3 || exit 1
echo ok > $O/done
