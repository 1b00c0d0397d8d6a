# Round-6 A/B: the pipeline's extractor contexts with (default) and without (CWT_PIPE_CONV_OCC=0)
# the layer1-3 conv plans measured beside a resident 59-CU grid; interleaved, driver's step counts.
set -u
OUT=gpurun_out/r6occab
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "pipeline or validate_transformer" > $OUT/pytest.txt 2>&1 || { echo "pytest rc=$?"; exit 1; }
echo "pytest ok"
for i in 1 2 3; do
  for occ in 0 59; do
    CWT_PIPE_CONV_OCC=$occ timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --exact-steps 0 --x3-steps 0 --pair-steps 0 > $OUT/bench_occ${occ}_r$i.json 2> $OUT/bench_occ${occ}_r$i.err || { echo "bench occ$occ r$i rc=$?"; exit 1; }
    echo "bench occ$occ r$i ok"
  done
done
