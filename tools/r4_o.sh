#!/bin/bash
# Round 4, box o: exact-fp32 (f32d) plan sweep over the variant heads' GEMM shapes (MMN
# WeightAverage forward and backward), and the MatchNet/DeTr backward tests at the final grid.
set -u
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r4o
mkdir -p $O
T="python -u -m pytest -x --timeout 300 --timeout-method thread"
timeout -k 10 400 $T -q tests/test_gpu_match_bwd.py tests/test_gpu_detr_bwd.py > $O/tests_bwd.log 2>&1 || exit $?
timeout -k 10 500 python -u tools/conv_s_sweep.py --prec 0 --vars 0,1,2,4 --configs 0:60:1 --out r4o/sweep_heads_f32d.json > $O/sweep_heads.log 2>&1 || exit $?
CWT_GEMM_F32D=2 timeout -k 10 200 python -u tools/time_match.py 1 5 > $O/time_match_f32d2.json 2> $O/time_match_f32d2.err || exit $?
timeout -k 10 200 python -u tools/time_match.py 1 5 > $O/time_match.json 2> $O/time_match.err || exit $?
echo done
