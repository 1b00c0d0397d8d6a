#!/bin/bash
# Round-4 operating points: configs #3, #4, #5 on the final build.
set -u
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r4final/configs
mkdir -p $O
timeout -k 10 300 python -u bench.py --shot 5 --steps 30 --exact-steps 0 --pair-steps 0 > $O/bench_shot5.json 2> $O/bench_shot5.err || exit $?
timeout -k 10 300 python -u bench.py --train --layers 101 --size 641 --steps 30 --exact-steps 0 --pair-steps 0 > $O/bench_train641.json 2> $O/bench_train641.err || exit $?
timeout -k 10 300 python -u bench.py --shot 5 --layers 101 --size 641 --conv-dtype bf16 --steps 20 --exact-steps 0 --pair-steps 0 > $O/bench_c5.json 2> $O/bench_c5.err || exit $?
echo done
