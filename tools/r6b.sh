set -u
mkdir -p gpurun_out/r6b
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_adapt_persist.py tests/test_gpu_tail.py "tests/test_gpu_parity.py::test_validate_transformer_vs_reference" "tests/test_gpu_parity.py::test_validate_transformer_pipelined_vs_reference" tests/test_gpu_detr_bwd.py tests/test_gpu_match_bwd.py > gpurun_out/r6b/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --profile-json gpurun_out/r6b/prof.json > gpurun_out/r6b/bench.json 2> gpurun_out/r6b/bench.err
echo "bench rc=$?"
