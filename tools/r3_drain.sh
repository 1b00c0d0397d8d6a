#!/bin/bash
# Pipeline drain A/B: the burst's last episode's inner loop on the whole-chip geometry
# (CWT_PIPE_DRAIN=1, default) against the pipeline geometry (=0), driver-like bench (20 steps,
# 5 warm-up), three interleaved pairs; pipeline tests first.
set -u
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/drain
timeout -k 10 400 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 -p no:cacheprovider > gpurun_out/drain/tests.txt 2>&1 || { tail -30 gpurun_out/drain/tests.txt; exit 1; }
tail -2 gpurun_out/drain/tests.txt
for rep in 1 2 3; do
  for d in 0 1; do
    tag=d${d}_$rep
    CWT_PIPE_DRAIN=$d timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --exact-steps 0 > gpurun_out/drain/b_$tag.json 2>gpurun_out/drain/b_$tag.err || exit 1
    python -c "import json; d=json.loads(open('gpurun_out/drain/b_$tag.json').read().strip().splitlines()[-1]); print('$tag', d['value'], d['roofline']['kernel'][:26], d['roofline']['avg_launch_ms'])" | tee -a gpurun_out/drain/summary.txt
  done
done
