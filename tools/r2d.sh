set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_adapt_persist.py -m gpu > gpurun_out/persist.log 2>&1 || { echo persist-fail; tail -30 gpurun_out/persist.log; exit 1; }
tail -1 gpurun_out/persist.log
for R in 2 4 8 16; do for SL in 0 1 4; do
  echo "R=$R sleep=$SL $(CWT_ADAPT_PR=$R CWT_ADAPT_SLEEP=$SL CWT_ADAPT_DBG=32 timeout -k 10 120 python tools/persist_stamps.py 1 473 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['loop per step (realtime)'], d['last adds issued -> first complete'], d['last adds issued -> last complete'], d['step work per workgroup min/median/max'])")" || exit 1
done; done
