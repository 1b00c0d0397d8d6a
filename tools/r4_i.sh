#!/bin/bash
# Round 4, box i: persistent CenterPivotConv4d tile schedules (CWT_CP4D_ORDER 0/1/2): parity and
# kernel stats; the L2 hit counts of each; WeightAverage / readout GEMMs on conv_igemm_f32d (A/B).  Tail with P1 tokens prefetched / reused in P4.
set -u
export TMPDIR=/tmp
O=gpurun_out/r4i
mkdir -p $O
T="python -u -m pytest -x --timeout 300 --timeout-method thread"
timeout -k 10 400 $T -v tests/test_gpu_match.py tests/test_gpu_detr.py tests/test_gpu_heads.py > $O/tests_match.log 2>&1 || exit $?
timeout -k 10 300 $T -v tests/test_gpu_tail.py > $O/tests_tail.log 2>&1 || exit $?
timeout -k 10 120 python -u tools/tail_stamps.py 60 20 > $O/tail_stamps.json 2> $O/tail_stamps.err || exit $?
CWT_TAIL_G=64 timeout -k 10 120 python -u tools/tail_stamps.py 60 20 > $O/tail_stamps_g64.json 2> $O/tail_stamps_g64.err || exit $?
cd /tmp && R=$GRAFT_REPO_ROOT
for v in 0 1 2; do
  export CWT_CP4D_ORDER=$v
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_o$v -o run -- \
    python -u $R/tools/time_match.py 1 3 > $R/$O/time_o$v.json 2> $R/$O/time_o$v.err || exit $?
  timeout -s KILL 120 rocprofv3 --kernel-trace --kernel-include-regex cp4d --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv \
    -d $R/$O/pmc_o$v -o run -- python -u $R/tools/time_match.py 1 1 > $R/$O/pmc_o$v.log 2>&1 || exit $?
done
cd $R
CWT_GEMM_F32D=0 timeout -k 10 200 python -u tools/time_match.py 1 5 > $O/time_gemm_old.json 2> $O/time_gemm_old.err || exit $?
timeout -k 10 200 python -u tools/time_match.py 1 5 > $O/time_gemm_f32d.json 2> $O/time_gemm_f32d.err || exit $?
for v in p0f1 p1f1 p0f0 p0f1 p1f1 p0f0; do
  CWT_PIPE_ADAPT_PRIO=${v:1:1} CWT_FUSED_TAIL=${v:3:1} timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 \
    --exact-steps 0 --pair-steps 0 --no-cpu-baseline >> $O/bench_$v.jsonl 2>> $O/bench_ab.err || exit $?
done
echo done
