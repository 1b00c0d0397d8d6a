set -u
OUT=gpurun_out/r6h
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_batch.py "tests/test_gpu_parity.py::test_validate_transformer_vs_reference" "tests/test_gpu_parity.py::test_validate_transformer_pipelined_vs_reference" > $OUT/pytest.log 2>&1 || { echo "pytest rc=$?"; exit 1; }
for r in 1 2; do
  for sp in 0 1; do
    CWT_PIPE_DRAIN_SPLIT=$sp timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --exact-steps 0 --x3-steps 0 --pair-steps 0 > $OUT/bench_split${sp}_r$r.json 2> $OUT/bench_split${sp}_r$r.err || { echo "bench rc=$?"; exit 1; }
  done
done
echo done
