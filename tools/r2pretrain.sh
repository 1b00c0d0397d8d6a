# stage-1 pretraining: kernel + whole-step parity tests against the oracle, then a bench and its profile
set -u
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_pretrain_ops.py -m gpu -x -v -s -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pretrain_ops.log 2>&1
rc=$?; tail -8 gpurun_out/pretrain_ops.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_pretrain.py -m gpu -x -v -s -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pretrain_tests.log 2>&1
rc=$?; grep -E "worst|PASS|FAIL|Error" gpurun_out/pretrain_tests.log | head -20; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --pretrain --steps ${PT_STEPS:-8} --warmup 2 ${PT_EXTRA:-} > gpurun_out/bench_pretrain.json 2> gpurun_out/bench_pretrain.err
rc=$?; tail -2 gpurun_out/bench_pretrain.json; tail -3 gpurun_out/bench_pretrain.err; exit $rc
