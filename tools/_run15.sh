set -o pipefail
O=gpurun_out/rehearse; mkdir -p $O
export TRAY_BENCH_BACKEND=gloo
for n in 2 4; do
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus $n --steps 16 --warmup 2 > $O/bench_n$n.log 2>&1 || exit 1
done
echo ok > $O/done
