#!/bin/bash
# Which PC-sampling configurations does rocprofv3 offer on this GPU? (listing only, no kernel runs)
set -u
O=gpurun_out/r9a; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 -L > $GRAFT_REPO_ROOT/$O/list.txt 2>&1
rc=$?; grep -i -n -A12 "pc.sampl\|PC Sampl" $GRAFT_REPO_ROOT/$O/list.txt | head -60; exit $rc
