#!/bin/bash
# Round 4, box aa: the rolling consensus kernels with an LDS-only step barrier (global loads and
# output stores stay in flight across steps) -- parity, then the layer timings (with the timing
# study legs) and MMN.forward.
set -u
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r4aa
mkdir -p $O
T="python -u -m pytest -x --timeout 300 --timeout-method thread"
timeout -k 10 300 $T -v -s tests/test_gpu_cp4d_roll.py > $O/tests_roll.log 2>&1 || exit $?
timeout -k 10 400 $T -q -s tests/test_gpu_match.py tests/test_gpu_match_bwd.py > $O/tests_match.log 2>&1 || exit $?
for d in 0 1 2 3; do
  CWT_CP4D_RDBG=$d timeout -k 10 120 python -u tools/time_cp4d.py 10 | sed "s/^{/{\"rdbg\": $d, /" >> $O/time_cp4d.jsonl 2>> $O/time.err || exit $?
done
for pf in 1 2; do
  CWT_CP4D_PF=$pf timeout -k 10 120 python -u tools/time_cp4d.py 10 | sed "s/^{/{\"pf\": $pf, /" >> $O/time_cp4d_pf.jsonl 2>> $O/time.err || exit $?
done
timeout -k 10 200 python -u tools/time_match.py >> $O/time_match.jsonl 2>> $O/time.err || exit $?
echo done
