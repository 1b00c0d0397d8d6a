#!/bin/bash
# Round 4, box t: the rolling-window CenterPivotConv4d kernel with four column slots (one
# barrier per step) -- parity, then the layer timings 3 vs 4 slots per columns-per-workgroup.
set -u
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r4t
mkdir -p $O
T="python -u -m pytest -x --timeout 300 --timeout-method thread"
timeout -k 10 300 $T -v -s tests/test_gpu_cp4d_roll.py > $O/tests_roll.log 2>&1 || exit $?
timeout -k 10 400 $T -q -s tests/test_gpu_match.py tests/test_gpu_match_bwd.py > $O/tests_match.log 2>&1 || exit $?
for ns in 4 3 4 3; do
  for wc in 30 20; do
    CWT_CP4D_NS=$ns CWT_CP4D_WC=$wc timeout -k 10 120 python -u tools/time_cp4d.py | sed "s/^{/{\"ns\": $ns, /" >> $O/time_cp4d.jsonl 2>> $O/time.err || exit $?
  done
done
for v in 1 0; do
  CWT_CP4D_ROLL=$v timeout -k 10 200 python -u tools/time_match.py >> $O/time_match_roll$v.jsonl 2>> $O/time.err || exit $?
done
echo done
