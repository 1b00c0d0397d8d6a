# Round-6 GPU test suite + smoke on the current tree (one process each, own time limits).
set -u
OUT=gpurun_out/r6t
mkdir -p $OUT
timeout -k 10 300 python -u __graft_entry__.py smoke > $OUT/smoke.txt 2>&1 || { echo "smoke rc=$?"; exit 1; }
echo "smoke ok"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1 || { echo "pytest rc=$?"; exit 1; }
echo "pytest ok"
