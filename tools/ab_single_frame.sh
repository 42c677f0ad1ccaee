#!/bin/bash
# A/B of the chunk-reservation settings in one-frame launches (the drop-in tray_render shape).
#   tools/build_variants.sh base "" lt1 "-DTRAY_LATE_TAKES=1u" lt2 "-DTRAY_LATE_TAKES=2u" wc8 "-DTRAY_WAVE_CHUNKS=8" wc4 "-DTRAY_WAVE_CHUNKS=4"
set -u
O=gpurun_out/single; mkdir -p $O
V=""; for v in base lt1 lt2 wc8 wc4; do V="$V $v=tray_amd/build/variants/$v/libtray_amd.so"; done
timeout -k 10 300 python3 tools/ab_bench.py --config c2 --passes 1 --rounds 15 $V > $O/ab_c2_f1.jsonl 2>$O/err1 || exit 1
timeout -k 10 300 python3 tools/ab_bench.py --config c1 --passes 1 --rounds 15 $V > $O/ab_c1_f1.jsonl 2>$O/err2 || exit 1
timeout -k 10 300 python3 tools/ab_bench.py --config c3 --passes 1 --rounds 3 $V > $O/ab_c3_f1.jsonl 2>$O/err3 || exit 1
echo ok > $O/done
