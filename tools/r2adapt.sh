# persistent inner loop: correctness (persist vs per-step kernel, reference episodes), stamps, bench
set -u
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_adapt_persist.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/adapt_tests.log 2>&1
rc=$?; tail -2 gpurun_out/adapt_tests.log; [ $rc -ne 0 ] && exit $rc
CWT_ADAPT_DBG=32 timeout -k 10 120 python -u tools/persist_stamps.py 1 473 > gpurun_out/stamps_r2b.log 2>&1
rc=$?; tail -20 gpurun_out/stamps_r2b.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_adapt.json 2> gpurun_out/bench_adapt.err
rc=$?; python -c "import json;d=json.loads(open('gpurun_out/bench_adapt.json').read().strip().splitlines()[-1]);print(d['value'],d['sequential'],d['roofline']['avg_launch_ms'],d['phases_roofline']['inner_loop'] if 'inner_loop' in d.get('phases_roofline',{}) else '')"; exit $rc
