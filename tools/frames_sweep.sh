mkdir -p gpurun_out/fsweep
B="timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-e2e --no-single"
for r in 1 2 3; do
  for cfg in "--passes 16" "--passes 20" "--passes 10" "--passes 20 --frames-in-flight 1" "--passes 7 --frames-in-flight 3"; do
    $B $cfg > gpurun_out/fsweep/o.txt 2>&1 || exit 1
    echo "$r $cfg $(grep '^{' gpurun_out/fsweep/o.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')" >> gpurun_out/fsweep/res.txt
  done
done
