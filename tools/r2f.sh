set -o pipefail
mkdir -p gpurun_out
for SH in 1 5; do for P in 0 1 2; do
  echo "shot=$SH persist=$P $(CWT_ADAPT_PERSIST=$P timeout -k 10 200 python bench.py --steps 20 --warmup 3 --shot $SH --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['phases_ms_per_step'])")" || exit 1
done; done
echo "R101 641 train $(timeout -k 10 200 python bench.py --steps 10 --warmup 2 --train --layers 101 --size 641 --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['phases_ms_per_step'])")"
echo "inflight4 $(timeout -k 10 200 python bench.py --steps 10 --warmup 2 --inflight 4 --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['phases_ms_per_step'])")"
echo "inflight4 step $(CWT_ADAPT_PERSIST=0 timeout -k 10 200 python bench.py --steps 10 --warmup 2 --inflight 4 --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['phases_ms_per_step'])")"
