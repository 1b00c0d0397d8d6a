#!/bin/bash
# Round 4, box z: re-check of the tidied consensus kernels (parity), then the inner loop's
# replica count (CWT_ADAPT_PR: rows the per-step partial sums are spread over) in the pipeline --
# the driver's bench command, interleaved.
set -u
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r4z
mkdir -p $O
T="python -u -m pytest -x --timeout 300 --timeout-method thread"
timeout -k 10 300 $T -q -s tests/test_gpu_cp4d_roll.py tests/test_gpu_match.py tests/test_gpu_match_bwd.py > $O/tests.log 2>&1 || exit $?
for r in 8 4 16 2 8 4 16 2; do
  CWT_ADAPT_PR=$r timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --exact-steps 0 --pair-steps 0 >> $O/bench_pr$r.jsonl 2>> $O/bench.err || exit $?
done
echo done
