set -u
mkdir -p gpurun_out/r6g
timeout -k 10 300 python -u __graft_entry__.py smoke > gpurun_out/r6g/smoke.log 2>&1 || { echo "smoke rc=$?"; exit 1; }
echo "smoke ok"
timeout -k 10 1500 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider -rf > gpurun_out/r6g/pytest_gpu.log 2>&1
echo "pytest rc=$?"
