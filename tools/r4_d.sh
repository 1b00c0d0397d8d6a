#!/bin/bash
# Round 4, box d: new kernels' parity (one-launch tail, two-register-unit inner loop, MFMA 4-D
# consensus, f32d conv), episode parity, f32d plan sweep, MMN timing A/B, the driver's bench
# command and its rocprofv3 stats.
set -u
export TMPDIR=/tmp
O=gpurun_out/r4d
mkdir -p $O
T="python -u -m pytest -x --timeout 300 --timeout-method thread"
timeout -k 10 300 $T -v tests/test_gpu_tail.py > $O/tests_tail.log 2>&1 || exit $?
timeout -k 10 600 $T -v tests/test_gpu_adapt_persist.py > $O/tests_persist.log 2>&1 || exit $?
timeout -k 10 400 $T -v tests/test_gpu_match.py > $O/tests_match.log 2>&1 || exit $?
timeout -k 10 600 $T -q tests/test_gpu_conv_s.py -k "f32d" > $O/tests_f32d.log 2>&1 || exit $?
timeout -k 10 600 $T -v tests/test_gpu_parity.py -k "exact_fp32 or episode_vs_reference" tests/test_gpu_batch.py tests/test_gpu_pretrain.py::test_pretrain_checkpoint_lr_is_post_step > $O/tests.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/conv_s_sweep.py --prec 0 --vars 0,1,2,4 --configs 50:473:2 --out r4d/sweep_f32d.json > $O/sweep_f32d.log 2>&1 || exit $?
CWT_CP4D_MFMA=0 timeout -k 10 200 python -u tools/time_match.py 1 5 > $O/time_match_scalar.json 2> $O/time_match_scalar.err || exit $?
timeout -k 10 200 python -u tools/time_match.py 1 5 > $O/time_match_mfma.json 2> $O/time_match_mfma.err || exit $?
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python -u bench.py --steps 20 --warmup 5 > $O/bench_prof.json 2> $O/bench_prof.err || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_match -o run -- \
  python -u tools/time_match.py 1 5 > $O/time_match_prof.json 2> $O/time_match_prof.err || exit $?
echo done
