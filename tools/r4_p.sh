#!/bin/bash
# Round 4, box p: WeightAverage on the f32d GEMMs with the measured plans (parity + MMN timing).
set -u
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r4p
mkdir -p $O
T="python -u -m pytest -x --timeout 300 --timeout-method thread"
timeout -k 10 400 $T -q tests/test_gpu_match.py tests/test_gpu_match_bwd.py tests/test_gpu_detr.py tests/test_gpu_detr_bwd.py > $O/tests.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/time_match.py 1 5 > $O/time_match.json 2> $O/time_match.err || exit $?
CWT_GEMM_F32D=0 timeout -k 10 200 python -u tools/time_match.py 1 5 > $O/time_match_gemm0.json 2> $O/time_match_gemm0.err || exit $?
echo done
