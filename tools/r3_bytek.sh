#!/bin/bash
# Byte kernels of the extractor (stem conv1 on the f32 MFMA, 8-channel PPM row pass, two-output
# max-pool): extraction parity tests, then the per-launch A/B against the previous forms.
set -u
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/bytek
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shapes.py tests/test_gpu_bf16.py tests/test_gpu_bn_train.py tests/test_gpu_batch.py -m gpu -x -q --timeout 300 -p no:cacheprovider > gpurun_out/bytek/tests.txt 2>&1 || { tail -30 gpurun_out/bytek/tests.txt; exit 1; }
tail -3 gpurun_out/bytek/tests.txt
for i in 1 2; do
  CWT_STEM_VALU=1 CWT_MAXPOOL1=1 timeout -k 10 120 python -u tools/time_extract.py --tag old >> gpurun_out/bytek/time.jsonl || exit 1
  timeout -k 10 120 python -u tools/time_extract.py --tag new >> gpurun_out/bytek/time.jsonl || exit 1
done
timeout -k 10 120 python -u tools/time_extract.py --tag new_bf16_641 --layers 101 --size 641 --n 6 >> gpurun_out/bytek/time.jsonl || exit 1
cat gpurun_out/bytek/time.jsonl
timeout -k 10 300 python -u bench.py --steps 60 --warmup 5 --no-cpu-baseline > gpurun_out/bytek/bench.json 2> gpurun_out/bytek/bench.err || exit 1
python -c "import json; d=json.loads(open('gpurun_out/bytek/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['sequential'], d['conv_stack']['roofline_frac'], d['phases_ms_per_step'])"
