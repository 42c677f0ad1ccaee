#!/bin/bash
set -u
O=gpurun_out/r8k; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; exit $rc
