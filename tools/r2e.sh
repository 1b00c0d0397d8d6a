set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q -s --timeout 120 --timeout-method thread tests/test_gpu_adapt_persist.py -m gpu > gpurun_out/persist.log 2>&1 || { echo persist-fail; tail -30 gpurun_out/persist.log; exit 1; }
grep "max rel" gpurun_out/persist.log; tail -1 gpurun_out/persist.log
for UC in 15 31; do for R in 4 8; do
  echo "UC=$UC R=$R $(CWT_ADAPT_UC=$UC CWT_ADAPT_PR=$R CWT_ADAPT_DBG=32 timeout -k 10 120 python tools/persist_stamps.py 1 473 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps(d))")" || exit 1
done; done
timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['phases_ms_per_step'])"
