#!/bin/bash
# Round-4 state of record, part 1: smoke + the whole -m gpu suite (one process, per-test timeout).
set -u
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=${O:-gpurun_out/r4final}
mkdir -p $O
timeout -k 10 300 python -u __graft_entry__.py smoke > $O/smoke.log 2>&1 || exit $?
timeout -k 10 1080 python -u -m pytest tests -m gpu -q -p no:cacheprovider -rf --timeout 300 --timeout-method thread \
  --durations=15 > $O/pytest_gpu.log 2>&1
rc=$?
tail -5 $O/pytest_gpu.log
exit $rc
