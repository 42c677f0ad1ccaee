#!/bin/bash
# Build kernel variants of libtray_amd.so for A/B timing (tools/ab_bench.py).
#   tools/build_variants.sh NAME "EXTRA HIPFLAGS" [NAME "FLAGS" ...]
set -e
cd "$(dirname "$0")/../tray_amd"
BASE="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-fast-math -mllvm -amdgpu-atomic-optimizer-strategy=None -fvisibility=hidden"
while [ $# -ge 2 ]; do
  NAME=$1; FLAGS=$2; shift 2
  OUT=build/variants/$NAME; mkdir -p $OUT
  pids=()
  for f in tray_kernel.hip tray_abi.hip tray_scale.hip; do
    /opt/rocm/bin/hipcc $BASE $FLAGS -c -o $OUT/$f.o csrc/$f & pids+=($!)
  done
  for f in tray_host.cpp tray_bvh.cpp; do
    /opt/rocm/bin/hipcc $BASE $FLAGS -x hip -c -o $OUT/$f.o csrc/$f & pids+=($!)
  done
  for p in "${pids[@]}"; do wait $p || { echo "compile failed: $NAME" >&2; exit 1; }; done
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o $OUT/libtray_amd.so $OUT/*.o
  echo "built $OUT/libtray_amd.so"
done
