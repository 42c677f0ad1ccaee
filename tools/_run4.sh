set -o pipefail
O=gpurun_out/spec4; mkdir -p $O
V=tray_amd/build/variants
timeout -k 10 300 python3 tools/ab_bench.py --config c2 --rounds 3 base=tray_amd/libtray_amd.so s8=$V/spec/libtray_amd.so@TRAY_SPEC=1 t4=$V/t4/libtray_amd.so@TRAY_SPEC=1 t12=$V/t12/libtray_amd.so@TRAY_SPEC=1 t8s16=$V/t8s16/libtray_amd.so@TRAY_SPEC=1 t8c4=$V/t8c4/libtray_amd.so@TRAY_SPEC=1 t12s16=$V/t12s16/libtray_amd.so@TRAY_SPEC=1 > $O/ab_c2.jsonl 2>&1 || exit 1
echo ok > $O/done
