#!/bin/bash
# One GPU session: smoke, parity tests, then (only if nothing crashed) a short bench with
# per-launch records.  Every GPU step has its own timeout; a crash/timeout ends the script.
set -u
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
STEPS=${STEPS:-10}
echo "== smoke $(date +%T)"
timeout -k 10 300 python -u __graft_entry__.py smoke 2>&1 | tee gpurun_out/smoke.log
rc=${PIPESTATUS[0]}
echo "smoke rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
echo "== pytest $(date +%T)"
timeout -k 10 900 python -u -m pytest ${PYTEST_PATHS:-tests} -m gpu -v -p no:cacheprovider -rf --timeout 300 --durations=0 ${PYTEST_ARGS:-} 2>&1 | tee gpurun_out/pytest_gpu.log
rc=${PIPESTATUS[0]}
echo "pytest rc=$rc"
if [ $rc -gt 1 ]; then exit $rc; fi
echo "== bench $(date +%T)"
timeout -k 10 400 python -u bench.py --steps $STEPS --warmup 2 ${BENCH_ARGS:-} --profile-json gpurun_out/prof.json > gpurun_out/bench.json 2> >(tee gpurun_out/bench.err >&2)
rc=$?
echo "bench rc=$rc"
cat gpurun_out/bench.json
exit $rc
