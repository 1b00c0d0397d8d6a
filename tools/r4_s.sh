#!/bin/bash
# Round 4, box s: the rolling-window CenterPivotConv4d kernel -- parity (one layer against a
# conv2d restatement, the MatchNet / MMN heads and their backward), then the layer timings per
# columns-per-workgroup setting and MMN.forward with / without it.
set -u
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r4s
mkdir -p $O
T="python -u -m pytest -x --timeout 300 --timeout-method thread"
timeout -k 10 300 $T -v -s tests/test_gpu_cp4d_roll.py > $O/tests_roll.log 2>&1 || exit $?
timeout -k 10 400 $T -q -s tests/test_gpu_match.py tests/test_gpu_match_bwd.py > $O/tests_match.log 2>&1 || exit $?
for wc in 20 60 30 15 10; do
  CWT_CP4D_WC=$wc timeout -k 10 120 python -u tools/time_cp4d.py >> $O/time_cp4d.jsonl 2>> $O/time.err || exit $?
done
for v in 1 0 1 0; do
  CWT_CP4D_ROLL=$v timeout -k 10 200 python -u tools/time_match.py >> $O/time_match_roll$v.jsonl 2>> $O/time.err || exit $?
done
echo done
