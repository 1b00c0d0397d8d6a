#!/bin/bash
# Round 4, box gg: MutualMatching with the transposition / branch-sum folded in (CWT_MM_FUSE=1)
# against the default -- parity of both (MatchNet / MMN / DeTr and their backward), then
# MMN.forward interleaved.
set -u
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r4gg
mkdir -p $O
T="python -u -m pytest -x --timeout 300 --timeout-method thread"
timeout -k 10 400 $T -q tests/test_gpu_match.py tests/test_gpu_match_bwd.py tests/test_gpu_detr.py tests/test_gpu_detr_bwd.py > $O/tests_fuse0.log 2>&1 || exit $?
CWT_MM_FUSE=1 timeout -k 10 400 $T -q tests/test_gpu_match.py tests/test_gpu_match_bwd.py tests/test_gpu_detr.py tests/test_gpu_detr_bwd.py > $O/tests_fuse1.log 2>&1 || exit $?
for v in 1 0 1 0; do
  CWT_MM_FUSE=$v timeout -k 10 200 python -u tools/time_match.py >> $O/time_match_fuse$v.jsonl 2>> $O/time.err || exit $?
done
echo done
