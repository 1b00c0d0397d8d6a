#!/bin/bash
# Round 4, box c: f32d conv parity + plan sweep, one-launch tail, pipeline batch, exact-fp32
# episodes, the driver's bench command and its rocprofv3 stats.
set -u
export TMPDIR=/tmp
O=gpurun_out/r4c
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_tail.py -k "one_launch or status_clean" > $O/tests_tail.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_conv_s.py -k "f32d" > $O/tests_f32d.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "exact_fp32 or episode_vs_reference" tests/test_gpu_batch.py tests/test_gpu_pretrain.py::test_pretrain_checkpoint_lr_is_post_step tests/test_gpu_adapt_persist.py > $O/tests.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/conv_s_sweep.py --prec 0 --vars 0,1,2,4 --configs 50:473:2 --out r4c/sweep_f32d.json > $O/sweep_f32d.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python -u bench.py --steps 20 --warmup 5 > $O/bench_prof.json 2> $O/bench_prof.err || exit $?
echo done
