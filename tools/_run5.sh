set -o pipefail
O=gpurun_out/prim; mkdir -p $O
for c in c2 c5; do timeout -k 10 120 python3 tools/primary_share.py tray_amd/build/variants/prim/libtray_amd.so --config $c >> $O/prim.jsonl 2>&1 || exit 1; done
echo ok > $O/done
