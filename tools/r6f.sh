set -u
mkdir -p gpurun_out/r6f
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_conv_s.py -k x6 tests/test_gpu_parity.py > gpurun_out/r6f/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --profile-json gpurun_out/r6f/prof.json > gpurun_out/r6f/bench.json 2> gpurun_out/r6f/bench.err
echo "bench rc=$?"
timeout -k 10 300 python -u tools/graph_extract.py > gpurun_out/r6f/graph_extract.log 2>&1
echo "graph rc=$?"
