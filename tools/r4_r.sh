#!/bin/bash
# Round 4, box r: the pipeline's overlapped drain (the burst's last loop beside the previous
# episode's loop and tail) -- pipeline parity, then the driver's bench command A/B, interleaved.
set -u
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r4r
mkdir -p $O
T="python -u -m pytest -x --timeout 300 --timeout-method thread"
timeout -k 10 400 $T -v -s tests/test_gpu_batch.py > $O/tests_batch.log 2>&1 || exit $?
for v in 1 0 1 0 1 0; do
  CWT_PIPE_DRAIN_OVERLAP=$v timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --exact-steps 0 --pair-steps 0 >> $O/bench_ov$v.jsonl 2>> $O/bench.err || exit $?
done
echo done
