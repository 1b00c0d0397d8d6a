set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_batch.py -m gpu -k pipeline > gpurun_out/pipe.log 2>&1 || { echo pipe-fail; tail -30 gpurun_out/pipe.log; exit 1; }
tail -1 gpurun_out/pipe.log
for A in "--pipeline 1" "--pipeline 2" "--pipeline 3" "--shot 5 --pipeline 2" "--layers 101 --size 641 --pipeline 1" "--layers 101 --size 641 --pipeline 2"; do
  echo "$A: $(timeout -k 10 200 python bench.py --steps 30 --warmup 4 $A --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['phases_ms_per_step'])")" || exit 1
done
