#!/bin/bash
# Round 4, box m: kernel statistics of the MMN head's forward + backward (tools/time_match.py).
set -u
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r4m
mkdir -p $O
cd /tmp && R=$GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o run -- \
  python -u $R/tools/time_match.py 1 3 > $R/$O/time_match.json 2> $R/$O/time_match.err || exit $?
echo done
