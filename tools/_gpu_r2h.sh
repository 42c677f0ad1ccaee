O=gpurun_out/r2h; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 180 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" > $O/status
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
L=tray_amd/libtray_amd.so
timeout -k 10 300 python3 tools/ab_bench.py --config c2 --rounds 9 old=$L@TRAY_RESOLVE_STAGED=0 staged=$L@TRAY_RESOLVE_STAGED=1 > $O/ab.jsonl 2>$O/ab.err; echo "ab rc=$?" >> $O/status
export TMPDIR=/tmp
for v in 0 1; do TRAY_RESOLVE_STAGED=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt$v -o kt --output-format csv -- python3 bench.py --steps 8 --warmup 0 --no-cpu-baseline --no-e2e --no-single --frames-in-flight 1 > $O/kt$v.log 2>&1; echo "kt$v rc=$?" >> $O/status; done
