set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "do_epoch" > gpurun_out/tr.log 2>&1 || { echo tr-fail; tail -30 gpurun_out/tr.log; exit 1; }
tail -1 gpurun_out/tr.log
for A in "" "--train" "--train --layers 101 --size 641" "--train --layers 101 --size 641 --pipeline 0" "--shot 5 --layers 101 --size 641 --conv-dtype bf16"; do
  echo "$A: $(timeout -k 10 300 python bench.py --steps 20 --warmup 3 $A --no-cpu-baseline 2>gpurun_out/b.err | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['phases_ms_per_step'], d['sequential'])")" || { tail -20 gpurun_out/b.err; exit 1; }
done
