# conv main-loop variants: correctness (every plan vs a float64 conv), then the plan sweeps
set -u
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_conv_s.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/conv_s_tests.log 2>&1
rc=$?; tail -2 gpurun_out/conv_s_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u tools/conv_s_sweep.py --configs 50:473:2,50:473:6,101:641:2 --vars 0,1,2,4 --out sweep_x3s_r2.json > gpurun_out/sweep_x3s_r2.log 2>&1
rc=$?; grep "sum over" gpurun_out/sweep_x3s_r2.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u tools/conv_s_sweep.py --prec 1 --configs 101:641:6,50:473:2 --vars 0,1,2,4 --out sweep_b16_r2.json > gpurun_out/sweep_b16_r2.log 2>&1
rc=$?; grep "sum over" gpurun_out/sweep_b16_r2.log; exit $rc
