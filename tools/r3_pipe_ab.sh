#!/bin/bash
# A/B of the pipeline's inner-loop geometry (units per workgroup on the adapt context)
set -o pipefail
O=${1:-gpurun_out/r3j}
mkdir -p $O
for u in 2 1 2 1; do
  CWT_PIPE_ADAPT_UNITS=$u timeout -k 10 200 python -u bench.py --steps 60 --no-cpu-baseline --exact-steps 0 >> $O/pipe_upw$u.jsonl 2>> $O/pipe.err || exit 1
done
