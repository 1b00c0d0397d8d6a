#!/bin/bash
# round-3 operating points: configs #3, #4, #5 on the current build
set -o pipefail
O=${1:-gpurun_out/r3l}
mkdir -p $O
timeout -k 10 300 python -u bench.py --shot 5 --steps 30 --exact-steps 0 > $O/bench_shot5.json 2> $O/bench_shot5.err || exit 1
timeout -k 10 300 python -u bench.py --train --layers 101 --size 641 --steps 30 --exact-steps 0 > $O/bench_train641.json 2> $O/bench_train641.err || exit 1
timeout -k 10 300 python -u bench.py --shot 5 --layers 101 --size 641 --conv-dtype bf16 --steps 20 --exact-steps 0 > $O/bench_c5.json 2> $O/bench_c5.err || exit 1
