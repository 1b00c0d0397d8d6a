# stage-1 pretraining: parity tests against the oracle
set -u
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_pretrain.py -m gpu -x -v -s -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pretrain_tests.log 2>&1
rc=$?; tail -30 gpurun_out/pretrain_tests.log; exit $rc
