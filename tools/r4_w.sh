#!/bin/bash
# Round 4, box w: kernel summary of MMN.forward at 473^2 (where the 5.9 ms go).
set -u
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r4w
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o mmn -- python3 -u tools/prof_mmn.py 10 > $O/prof.log 2>&1 || exit $?
echo done
