#!/bin/bash
# Round 4, box n: MFMA weight gradients of the 4-D consensus (parity + MMN train-step timing, the
# scalar form as A/B), two-stage column sums.
set -u
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r4n
mkdir -p $O
T="python -u -m pytest -x --timeout 300 --timeout-method thread"
timeout -k 10 400 $T -v -s tests/test_gpu_match_bwd.py tests/test_gpu_detr_bwd.py > $O/tests_bwd.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/time_match.py 1 5 > $O/time_match.json 2> $O/time_match.err || exit $?
CWT_DGRAD_SCALAR=1 timeout -k 10 200 python -u tools/time_match.py 1 3 > $O/time_match_dscalar.json 2> $O/time_match_dscalar.err || exit $?
cd /tmp && R=$GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o run -- \
  python -u $R/tools/time_match.py 1 3 > $R/$O/time_match_prof.json 2> $R/$O/time_match_prof.err || exit $?
echo done
