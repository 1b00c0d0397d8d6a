#!/bin/bash
# rocprofv3 kernel trace + stats of a short bench run (same command as the bench line).
set -u
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/prof_r1}
mkdir -p $OUT
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- \
  python -u bench.py --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/bench.json 2> $OUT/bench.err
rc=$?
echo "rocprof rc=$rc"
cat $OUT/bench.json
find $OUT -name "*stats*" | head
exit $rc
