#!/bin/bash
# Round 4, box q: the streamed inner loop with the first unit resident (<6>) -- parity against the
# step launches, and the 5-shot 641^2 loop alone A/B (<6> vs <3>), interleaved.
set -u
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r4q
mkdir -p $O
T="python -u -m pytest -x --timeout 300 --timeout-method thread"
timeout -k 10 400 $T -v -s tests/test_gpu_adapt_persist.py > $O/tests_persist.log 2>&1 || exit $?
for v in 1 0 1 0; do
  CWT_ADAPT_RES1=$v timeout -k 10 120 python -u tools/time_adapt.py 5 641 20 >> $O/time_adapt_res$v.jsonl 2>> $O/time_adapt.err || exit $?
done
echo done
