set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_adapt_persist.py -m gpu > gpurun_out/persist.log 2>&1 || { echo persist-fail; tail -30 gpurun_out/persist.log; exit 1; }
tail -2 gpurun_out/persist.log
CWT_ADAPT_DBG=32 timeout -k 10 120 python tools/persist_stamps.py 1 473 || exit 1
timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['phases_ms_per_step'])"
