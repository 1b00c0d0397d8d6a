#!/bin/bash
# (Record of the round-3 A/B in profiles/r3/sweeps_rejected/splitk_inlaunch_*.  The in-launch combine was
# slower and was removed afterwards, with its CWT_SPLITK_EPI switch.)
# In-launch split-K combine of conv_x3s (the tile's last arriver sums the partials): per-plan
# parity (every split-K plan), extraction parity, then A/B against the separate epilogue launch
# (CWT_SPLITK_EPI=1): extractor per-launch sums and the default bench.
set -u
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/splitk
timeout -k 10 700 python -u -m pytest tests/test_gpu_conv_s.py tests/test_gpu_parity.py tests/test_gpu_bf16.py tests/test_gpu_shapes.py -m gpu -x -q --timeout 300 -p no:cacheprovider > gpurun_out/splitk/tests.txt 2>&1 || { tail -40 gpurun_out/splitk/tests.txt; exit 1; }
tail -2 gpurun_out/splitk/tests.txt
for i in 1 2; do
  CWT_SPLITK_EPI=1 timeout -k 10 120 python -u tools/time_extract.py --tag epi --match splitk >> gpurun_out/splitk/time.jsonl || exit 1
  timeout -k 10 120 python -u tools/time_extract.py --tag inlaunch --match splitk >> gpurun_out/splitk/time.jsonl || exit 1
done
CWT_SPLITK_EPI=1 timeout -k 10 200 python -u tools/time_extract.py --tag epi_101_641_6 --layers 101 --size 641 --n 6 --match splitk >> gpurun_out/splitk/time.jsonl || exit 1
timeout -k 10 200 python -u tools/time_extract.py --tag inlaunch_101_641_6 --layers 101 --size 641 --n 6 --match splitk >> gpurun_out/splitk/time.jsonl || exit 1
cat gpurun_out/splitk/time.jsonl
for rep in 1 2; do
  for e in 1 0; do
    CWT_SPLITK_EPI=$e timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --exact-steps 0 > gpurun_out/splitk/b_${e}_${rep}.json 2>gpurun_out/splitk/b_${e}_${rep}.err || exit 1
    python -c "import json; d=json.loads(open('gpurun_out/splitk/b_${e}_${rep}.json').read().strip().splitlines()[-1]); print('epi=$e rep $rep', d['value'], d['sequential']['value'], d['conv_stack']['roofline_frac'], d['conv_roofline']['avg_launch_ms'])" | tee -a gpurun_out/splitk/summary.txt
  done
done
