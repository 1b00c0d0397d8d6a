# Round-6 check: the tail's counters by constant index (no promoted 48 KB / 24 KB of LDS):
# the tail / loop / parity / batch tests, then the default bench.
set -u
OUT=gpurun_out/r6tailfix
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_tail.py tests/test_gpu_adapt_persist.py tests/test_gpu_parity.py tests/test_gpu_batch.py tests/test_gpu_edges.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.txt 2>&1 || { echo "pytest rc=$?"; exit 1; }
echo "pytest ok"
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { echo "bench rc=$?"; exit 1; }
echo "bench ok"
