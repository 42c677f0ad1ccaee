#!/bin/bash
# Final-tree check: the driver's round-end sequence (smoke, then the default bench line).
set -u
O=gpurun_out/r8l; mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
timeout -k 10 600 python -u bench.py > $O/bench.log 2>&1
rc=$?; tail -1 $O/bench.log; exit $rc
