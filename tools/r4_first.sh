#!/bin/bash
# Round 4, first box: f32 conv plan sweep, the driver's bench command, and its rocprofv3 stats.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r4a
timeout -k 10 300 python -u tools/conv_f32_sweep.py --configs 50:473:2 --out r4a/conv_f32_sweep.json > gpurun_out/r4a/sweep_f32.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r4a/bench.json 2> gpurun_out/r4a/bench.err || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4a/prof -o run -- \
  python -u bench.py --steps 20 --warmup 5 > gpurun_out/r4a/bench_prof.json 2> gpurun_out/r4a/bench_prof.err || exit $?
echo done
