# Round-6 A/B: layer4 and the bottleneck on 256x256 tiles (CWT_X6_BIGTILE=1) against the plan table, interleaved.
set -u
OUT=gpurun_out/r6bigab
mkdir -p $OUT
CWT_X6_BIGTILE=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "validate_transformer" > $OUT/pytest.txt 2>&1 || { echo "pytest rc=$?"; exit 1; }
echo "pytest ok"
for i in 1 2 3; do
  for occ in 0 1; do
    CWT_X6_BIGTILE=$occ timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --exact-steps 0 --x3-steps 0 --pair-steps 0 > $OUT/bench_occ${occ}_r$i.json 2> $OUT/bench_occ${occ}_r$i.err || { echo "bench occ$occ r$i rc=$?"; exit 1; }
    echo "bench occ$occ r$i ok"
  done
done
