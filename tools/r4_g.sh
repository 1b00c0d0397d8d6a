#!/bin/bash
# Round 4, box g: persistent CenterPivotConv4d kernels (parity, A/B timing, kernel stats), tail tests.
set -u
export TMPDIR=/tmp
O=gpurun_out/r4g
mkdir -p $O
T="python -u -m pytest -x --timeout 300 --timeout-method thread"
timeout -k 10 400 $T -v tests/test_gpu_match.py > $O/tests_match.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/time_match.py 1 5 > $O/time_match_persist.json 2> $O/time_match_persist.err || exit $?
CWT_CP4D_PERSIST=0 timeout -k 10 200 python -u tools/time_match.py 1 5 > $O/time_match_tile.json 2> $O/time_match_tile.err || exit $?
cd /tmp && R=$GRAFT_REPO_ROOT && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_match -o run -- \
  python -u $R/tools/time_match.py 1 5 > $R/$O/time_match_prof.json 2> $R/$O/time_match_prof.err || exit $?
echo done
