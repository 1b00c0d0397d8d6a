set -u
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_pretrain_ops.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pt_ops.txt 2>&1
rc=$?; tail -1 gpurun_out/pt_ops.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --pretrain --steps 8 --warmup 2 --no-cpu-baseline > gpurun_out/bench_pretrain.json 2>/dev/null || exit 1
python -c "import json;d=json.loads(open('gpurun_out/bench_pretrain.json').read().strip().splitlines()[-1]);print('pretrain', d['value'], d['ms_per_step'])"
for k in 2 3; do timeout -k 10 200 python -u bench.py --pipeline $k --no-cpu-baseline > gpurun_out/pipe_$k.json 2>/dev/null || exit 1; python -c "import json;d=json.loads(open('gpurun_out/pipe_$k.json').read().strip().splitlines()[-1]);print('pipeline', $k, d['value'], d['roofline']['avg_launch_ms'])"; done
