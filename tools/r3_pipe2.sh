#!/bin/bash
# (Record of the round-3 A/B in profiles/r3/pipeline_ab/edges_units_streams.txt.  The burst-edge and
# second-adapt-stream variants measured slower and were removed afterwards; CWT_PIPE_ADAPT_UNITS=3 remains.)
# Pipeline A/B: burst edges (CWT_PIPE_EDGES), units per workgroup of the pipeline's inner loop
# (2 / 3) and adapt streams (1 / 2), default 1-shot R50 473 bench at the driver's 20 steps and at
# 60, interleaved, twice.  Then the stem conv1 forms (VALU vs f32 MFMA with gather prefetch).
set -u
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/pipe2
timeout -k 10 400 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 -p no:cacheprovider > gpurun_out/pipe2/tests.txt 2>&1 || { tail -30 gpurun_out/pipe2/tests.txt; exit 1; }
tail -2 gpurun_out/pipe2/tests.txt
CWT_PIPE_ADAPT_STREAMS=2 CWT_PIPE_ADAPT_UNITS=3 timeout -k 10 300 python -u -m pytest tests/test_gpu_batch.py -m gpu -x -q --timeout 200 -p no:cacheprovider > gpurun_out/pipe2/tests_s2u3.txt 2>&1 || { tail -30 gpurun_out/pipe2/tests_s2u3.txt; exit 1; }
tail -2 gpurun_out/pipe2/tests_s2u3.txt
for steps in 20 60; do
for rep in 1 2; do
  for cfg in "1 2 1" "0 2 1" "1 3 1" "1 3 2" "1 2 2"; do
    set -- $cfg
    tag=e$1_u$2_s$3_k${steps}_$rep
    CWT_PIPE_EDGES=$1 CWT_PIPE_ADAPT_UNITS=$2 CWT_PIPE_ADAPT_STREAMS=$3 timeout -k 10 200 python -u bench.py --steps $steps --warmup 5 --no-cpu-baseline --exact-steps 0 > gpurun_out/pipe2/b_$tag.json 2>gpurun_out/pipe2/b_$tag.err || exit 1
    python -c "import json,sys; d=json.loads(open('gpurun_out/pipe2/b_$tag.json').read().strip().splitlines()[-1]); print('$tag', d['value'], d['phases_ms_per_step'], d['roofline']['kernel'][:26], d['roofline']['avg_launch_ms'])" | tee -a gpurun_out/pipe2/summary.txt
  done
done
done
for i in 1 2; do
  CWT_STEM_VALU=1 timeout -k 10 120 python -u tools/time_extract.py --tag stem_valu --match stem >> gpurun_out/pipe2/time.jsonl || exit 1
  timeout -k 10 120 python -u tools/time_extract.py --tag stem_mfma_prefetch --match stem >> gpurun_out/pipe2/time.jsonl || exit 1
done
cat gpurun_out/pipe2/time.jsonl
