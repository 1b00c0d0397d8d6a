#!/bin/bash
# Round 4, box cc: the symmetric NeighConsensus branches on two streams -- parity (MatchNet /
# MMN / DeTr and their backward), then MMN.forward with / without (interleaved).
set -u
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r4cc
mkdir -p $O
T="python -u -m pytest -x --timeout 300 --timeout-method thread"
timeout -k 10 400 $T -q -s tests/test_gpu_match.py tests/test_gpu_match_bwd.py tests/test_gpu_detr.py tests/test_gpu_detr_bwd.py > $O/tests.log 2>&1 || exit $?
for v in 1 0 1 0; do
  CWT_MATCH_BRANCH_STREAMS=$v timeout -k 10 200 python -u tools/time_match.py >> $O/time_match_bs$v.jsonl 2>> $O/time.err || exit $?
done
echo done
