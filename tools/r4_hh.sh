#!/bin/bash
# Round 4, box hh: the DeTr backward case with the MutualMatching folds on / off (printed errors),
# and MMN.forward interleaved.
set -u
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r4hh
mkdir -p $O
T="python -u -m pytest --timeout 300 --timeout-method thread"
for v in 0 1; do
  CWT_MM_FUSE=$v timeout -k 10 300 $T -q -s tests/test_gpu_detr_bwd.py -k "test_detr_backward" > $O/tests_detr_fuse$v.log 2>&1
  echo "fuse$v rc=$?" >> $O/rc.txt
done
for v in 1 0 1 0; do
  CWT_MM_FUSE=$v timeout -k 10 200 python -u tools/time_match.py >> $O/time_match_fuse$v.jsonl 2>> $O/time.err || exit $?
done
echo done
