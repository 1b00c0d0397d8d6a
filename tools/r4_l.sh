#!/bin/bash
# Round 4, box l: DeTr head backward parity (test_gpu_detr_bwd.py), the MatchNet / MMN backward
# again, the forward tests of the heads (grad-enabled calls take the autograd path), and the
# MMN head timing (inference + the head's forward+backward).
set -u
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r4l
mkdir -p $O
T="python -u -m pytest -x --timeout 300 --timeout-method thread"
timeout -k 10 400 $T -v -s tests/test_gpu_detr_bwd.py > $O/tests_detr_bwd.log 2>&1 || exit $?
timeout -k 10 400 $T -v -s tests/test_gpu_match_bwd.py > $O/tests_match_bwd.log 2>&1 || exit $?
timeout -k 10 400 $T -q tests/test_gpu_match.py tests/test_gpu_detr.py tests/test_gpu_heads.py > $O/tests_heads.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/time_match.py 1 5 > $O/time_match.json 2> $O/time_match.err || exit $?
echo done
