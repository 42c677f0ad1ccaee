#!/bin/bash
# Kernel-trace stats and HBM counters of the default bench command (run on the
# GPU box from the repo root). Each rocprofv3 pass is its own run; --pmc passes
# never combine tracing domains.
#   usage: tools/profile_bench.sh <outdir> [bench.py args...]
set -u
OUT=${1:-gpurun_out/prof}; shift || true
ARGS=${*:-"--steps 16 --warmup 0 --no-cpu-baseline --no-e2e --no-single --frames-in-flight 1"}
export TMPDIR=/tmp
mkdir -p "$OUT"
# the device code these counters describe (bench.py only reuses them for the same code)
python3 -c "from tray_amd import _lib; print(_lib.code_object_sha256())" > "$OUT/code_object_sha256.txt" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o kt --output-format csv -- python3 bench.py $ARGS > "$OUT/kt.log" 2>&1 || exit 1
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --kernel-include-regex render_kernel -d "$OUT/$C" -o pmc --output-format csv -- python3 bench.py $ARGS > "$OUT/$C.log" 2>&1 || exit 1
done
echo done > "$OUT/status.txt"
