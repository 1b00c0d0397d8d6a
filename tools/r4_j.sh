#!/bin/bash
# Round 4, box j: the measured cp4d / GEMM defaults (MMN timing + kernel stats), and the
# pipeline's tail A/B: module path vs the one-launch tail at G = 64 / 32 / 16 (interleaved).
set -u
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r4j
mkdir -p $O
T="python -u -m pytest -x --timeout 300 --timeout-method thread"
timeout -k 10 400 $T -q tests/test_gpu_match.py tests/test_gpu_detr.py > $O/tests_match.log 2>&1 || exit $?
cd /tmp && R=$GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_match -o run -- \
  python -u $R/tools/time_match.py 1 5 > $R/$O/time_match.json 2> $R/$O/time_match.err || exit $?
cd $R
for v in f0 g64 g32 g16 f0 g64 g32 g16; do
  case $v in f0) E="CWT_FUSED_TAIL=0" ;; g64) E="CWT_FUSED_TAIL=1" ;; g32) E="CWT_TAIL_G=32" ;; g16) E="CWT_TAIL_G=16" ;; esac
  env $E timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --exact-steps 0 --pair-steps 0 --no-cpu-baseline \
    >> $O/bench_$v.jsonl 2>> $O/bench_ab.err || exit $?
done
echo done
