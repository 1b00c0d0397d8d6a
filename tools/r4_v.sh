#!/bin/bash
# Round 4, box v: the rolling-window CenterPivotConv4d kernels with a two-deep register prefetch
# (PF 2) against one-deep (PF 1) -- parity, the layer timings, MMN.forward.
set -u
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r4v
mkdir -p $O
T="python -u -m pytest -x --timeout 300 --timeout-method thread"
timeout -k 10 300 $T -v -s tests/test_gpu_cp4d_roll.py > $O/tests_roll.log 2>&1 || exit $?
timeout -k 10 400 $T -q -s tests/test_gpu_match.py tests/test_gpu_match_bwd.py > $O/tests_match.log 2>&1 || exit $?
for pf in 2 1 2 1; do
  CWT_CP4D_PF=$pf timeout -k 10 120 python -u tools/time_cp4d.py | sed "s/^{/{\"pf\": $pf, /" >> $O/time_cp4d.jsonl 2>> $O/time.err || exit $?
done
for v in 1 2 0; do
  CWT_CP4D_ROLL=$v timeout -k 10 200 python -u tools/time_match.py >> $O/time_match_roll$v.jsonl 2>> $O/time.err || exit $?
done
echo done
