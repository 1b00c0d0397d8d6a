#!/bin/bash
# Round 4, box dd: MutualMatching with per-pair channel vectors and a row-per-block apply --
# parity (MatchNet / MMN / DeTr and their backward), then MMN.forward and a kernel summary.
set -u
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=${O:-gpurun_out/r4dd}
mkdir -p $O
T="python -u -m pytest -x --timeout 300 --timeout-method thread"
timeout -k 10 400 $T -q -s tests/test_gpu_match.py tests/test_gpu_match_bwd.py tests/test_gpu_detr.py tests/test_gpu_detr_bwd.py > $O/tests.log 2>&1 || exit $?
for r in 1 2; do
  timeout -k 10 200 python -u tools/time_match.py >> $O/time_match.jsonl 2>> $O/time.err || exit $?
done
cd /tmp && R=$GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o mmn -- python3 -u $R/tools/prof_mmn.py 10 > $R/$O/prof.log 2>&1 || exit $?
echo done
