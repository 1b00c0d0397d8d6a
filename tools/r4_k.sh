#!/bin/bash
# Round 4, box k: MatchNet / MMN backward parity (test_gpu_match_bwd.py) and the forward tests
# of the same head (the autograd path now serves grad-enabled calls).
set -u
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r4k
mkdir -p $O
T="python -u -m pytest -x --timeout 300 --timeout-method thread"
timeout -k 10 400 $T -v -s tests/test_gpu_match_bwd.py > $O/tests_match_bwd.log 2>&1 || exit $?
timeout -k 10 400 $T -q tests/test_gpu_match.py tests/test_gpu_detr.py tests/test_gpu_heads.py > $O/tests_match.log 2>&1 || exit $?
echo done
