set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -s tests/test_gpu_adapt_persist.py -m gpu > gpurun_out/persist.log 2>&1 || { echo persist-fail; tail -30 gpurun_out/persist.log; exit 1; }
grep -E "max rel|PASS|FAIL" gpurun_out/persist.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_batch.py tests/test_gpu_shapes.py -m gpu > gpurun_out/parity2.log 2>&1; echo parity rc=$?; tail -3 gpurun_out/parity2.log
timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_persist.json 2> gpurun_out/bench_persist.err; echo bench rc=$?
CWT_ADAPT_PERSIST=0 timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_step.json 2>/dev/null; echo bench0 rc=$?
python -c "
import json
for f in ['bench_persist','bench_step']:
    d=json.load(open('gpurun_out/'+f+'.json')); print(f, d['value'], d['ms_per_step'], d['phases_ms_per_step'])
"
