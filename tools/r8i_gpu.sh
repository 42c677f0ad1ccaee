#!/bin/bash
# Round 5: does a collective after each launch starve behind the next persistent grid? (tools/comm_starve.py)
set -u
O=gpurun_out/r8i; mkdir -p $O
timeout -k 10 300 python3 tools/comm_starve.py --n 8 --comm-mb 155 --reserve 0,1,8 > $O/starve_n8_155.jsonl 2> $O/starve.err || exit 1
timeout -k 10 300 python3 tools/comm_starve.py --n 8 --comm-mb 22 --reserve 0,1,8 > $O/starve_n8_22.jsonl 2>> $O/starve.err || exit 1
timeout -k 10 300 python3 tools/comm_starve.py --n 1 --comm-mb 0.5 --reserve 0,1,8 --launches 4 > $O/starve_n1.jsonl 2>> $O/starve.err || exit 1
echo done > $O/done
