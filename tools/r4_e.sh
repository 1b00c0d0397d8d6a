#!/bin/bash
# Round 4, box e: tail (LDS-staged metrics) parity + phase stamps, 4-D consensus parity + timing,
# f32d plan table parity, batch tests, the driver's bench command.
set -u
export TMPDIR=/tmp
O=gpurun_out/r4e
mkdir -p $O
T="python -u -m pytest -x --timeout 300 --timeout-method thread"
timeout -k 10 300 $T -v tests/test_gpu_tail.py > $O/tests_tail.log 2>&1 || exit $?
timeout -k 10 120 python -u tools/tail_stamps.py 60 20 > $O/tail_stamps.json 2> $O/tail_stamps.err || exit $?
timeout -k 10 120 python -u tools/tail_stamps.py 81 20 > $O/tail_stamps81.json 2> $O/tail_stamps81.err || exit $?
timeout -k 10 400 $T -v tests/test_gpu_match.py > $O/tests_match.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/time_match.py 1 5 > $O/time_match_mfma.json 2> $O/time_match_mfma.err || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_match -o run -- \
  python -u tools/time_match.py 1 5 > $O/time_match_prof.json 2> $O/time_match_prof.err || exit $?
timeout -k 10 600 $T -v tests/test_gpu_parity.py -k "exact_fp32" > $O/tests_exact.log 2>&1 || exit $?
timeout -k 10 600 $T -v tests/test_gpu_batch.py > $O/tests_batch.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit $?
echo done
