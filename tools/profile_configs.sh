#!/bin/bash
# Counter profiles (kernel trace, HBM bytes, instruction mix) of the new code object for the
# configs given, so every bench line carries traffic and utilisation again.
#   usage: tools/profile_configs.sh c2 c1 ...
set -u
O=${O:-gpurun_out/prof}; mkdir -p $O
for c in "$@"; do
  bash tools/gpu_profile_all.sh $O/$c $c || { echo "profile $c failed"; exit 1; }
  echo "profiled $c"
done
