# A/B: persistent grid leaving 0 / 4 / 8 CUs to the other slot's resolve pass (bench shape)
O=gpurun_out/r2f; mkdir -p $O
for rep in 1 2; do for r in 0 4 8 2; do
TRAY_RESERVE_CUS=$r timeout -k 10 200 python3 bench.py --steps 24 --warmup 8 --no-cpu-baseline --no-e2e --no-single > $O/bench_r${r}_$rep.log 2>&1 || exit 1
done; done
echo ok > $O/status
