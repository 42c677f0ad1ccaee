set -o pipefail
O=gpurun_out/ground; mkdir -p $O
for c in c2 c5; do timeout -k 10 120 python3 tools/ground_share.py tray_amd/build/variants/ground/libtray_amd.so --config $c >> $O/ground.jsonl 2>&1 || exit 1; done
echo ok > $O/done
