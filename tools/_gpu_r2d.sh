# round-2 A/B: BVH width 8 vs 4, round-1 library; gloo rehearsal of the N=2 bench path
O=gpurun_out/r2d; mkdir -p $O
V=tray_amd/build/variants
timeout -k 10 300 python3 tools/ab_bench.py --config c2 --rounds 7 base=$V/base/libtray_amd.so r1=$V/r1/libtray_amd.so w8=$V/w8/libtray_amd.so w8n2=$V/w8n2/libtray_amd.so > $O/ab_c2.jsonl 2>$O/ab_c2.err || exit 1
timeout -k 10 300 python3 tools/ab_bench.py --config c5 --rounds 5 base=$V/base/libtray_amd.so w8=$V/w8/libtray_amd.so > $O/ab_c5.jsonl 2>$O/ab_c5.err || exit 1
TRAY_BENCH_BACKEND=gloo timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 8 --warmup 2 --no-cpu-baseline --no-e2e > $O/gloo2.log 2>&1; echo "gloo rc=$?" > $O/status
