#!/bin/bash
# Round 4, box y: rolling-window consensus kernels with coalesced output stores (D rows permuted
# so one store covers 4 consecutive b positions) and the COUT = 1 form's filters from scalar loads
# -- parity, then the layer timings and MMN.forward (with the COUT = 1 roll form on / off).
set -u
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r4y
mkdir -p $O
T="python -u -m pytest -x --timeout 300 --timeout-method thread"
timeout -k 10 300 $T -v -s tests/test_gpu_cp4d_roll.py > $O/tests_roll.log 2>&1 || exit $?
timeout -k 10 400 $T -q -s tests/test_gpu_match.py tests/test_gpu_match_bwd.py > $O/tests_match.log 2>&1 || exit $?
for d in 0 3 0; do
  CWT_CP4D_RDBG=$d timeout -k 10 120 python -u tools/time_cp4d.py 10 | sed "s/^{/{\"rdbg\": $d, /" >> $O/time_cp4d.jsonl 2>> $O/time.err || exit $?
done
for v in 2 1; do
  CWT_CP4D_ROLL=$v timeout -k 10 200 python -u tools/time_match.py >> $O/time_match_roll$v.jsonl 2>> $O/time.err || exit $?
done
echo done
