#!/bin/bash
# bench.py --config c1, alternating the in-tree library (on-chip pixel-pass sums) and HEAD's
# (FP64 sample-order sum for r = 16): is the timed-loop difference the change or the box?
set -u
O=gpurun_out/r9e${STEPS:-}; mkdir -p $O
for i in 1 2 3 4; do
  for V in new head; do
    if [ $V = head ]; then export TRAY_LIB=$PWD/tray_amd/build/variants/head/libtray_amd.so; else unset TRAY_LIB; fi
    timeout -k 10 200 python -u bench.py --config c1 --steps ${STEPS:-20} --no-cpu-baseline --no-e2e --no-single > $O/b_${V}_$i.log 2>&1 || { tail -5 $O/b_${V}_$i.log; exit 1; }
    tail -1 $O/b_${V}_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$V', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['plan']['acc_slots'])"
  done
done
