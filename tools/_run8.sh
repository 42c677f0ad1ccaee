set -o pipefail
mkdir -p gpurun_out/exec
timeout -k 10 60 ./tools/exec_half > gpurun_out/exec/exec_half.jsonl 2>&1 || exit 1
