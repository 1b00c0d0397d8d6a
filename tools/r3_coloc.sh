#!/bin/bash
# (Record of the round-3 A/B in profiles/r3/pipeline_ab/coloc.txt; the co-resident form was slower and
# was removed afterwards with its CWT_ADAPT_COLOC switch.)
# Loop / conv co-residency A/B: the pipeline's inner loop with one unit per workgroup under a
# 96-VGPR budget (adapt_persist_kernel<1, false, 5>, CWT_ADAPT_COLOC=1) so that a 64x64 conv
# workgroup fits beside it, against the default two-unit geometry and the plain one-unit form.
set -u
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/coloc
CWT_ADAPT_COLOC=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_adapt_persist.py tests/test_gpu_batch.py -m gpu -x -q --timeout 200 -p no:cacheprovider > gpurun_out/coloc/tests.txt 2>&1 || { tail -30 gpurun_out/coloc/tests.txt; exit 1; }
tail -2 gpurun_out/coloc/tests.txt
for rep in 1 2; do
  for cfg in "2 0" "1 0" "1 1"; do
    set -- $cfg
    tag=u$1_c$2_$rep
    CWT_PIPE_ADAPT_UNITS=$1 CWT_ADAPT_COLOC=$2 timeout -k 10 200 python -u bench.py --steps 60 --warmup 5 --no-cpu-baseline --exact-steps 0 > gpurun_out/coloc/b_$tag.json 2>gpurun_out/coloc/b_$tag.err || exit 1
    python -c "import json; d=json.loads(open('gpurun_out/coloc/b_$tag.json').read().strip().splitlines()[-1]); print('$tag', d['value'], d['sequential']['value'], d['phases_ms_per_step'], d['roofline']['kernel'][:26], d['roofline']['avg_launch_ms'])" | tee -a gpurun_out/coloc/summary.txt
  done
done
