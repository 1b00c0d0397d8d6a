#!/bin/bash
# Round 4, box f: tail at full-chip width (G = 256) with contiguous P5 pixel ranges: parity,
# phase stamps at G = 256 and 64, pipeline batch tests (adapt context at G = 64), the bench.
set -u
export TMPDIR=/tmp
O=gpurun_out/r4f
mkdir -p $O
T="python -u -m pytest -x --timeout 300 --timeout-method thread"
timeout -k 10 300 $T -v tests/test_gpu_tail.py > $O/tests_tail.log 2>&1 || exit $?
timeout -k 10 120 python -u tools/tail_stamps.py 60 20 > $O/tail_stamps.json 2> $O/tail_stamps.err || exit $?
CWT_TAIL_G=64 timeout -k 10 120 python -u tools/tail_stamps.py 60 20 > $O/tail_stamps_g64.json 2> $O/tail_stamps_g64.err || exit $?
CWT_TAIL_G=128 timeout -k 10 120 python -u tools/tail_stamps.py 60 20 > $O/tail_stamps_g128.json 2> $O/tail_stamps_g128.err || exit $?
timeout -k 10 120 python -u tools/tail_stamps.py 81 20 > $O/tail_stamps81.json 2> $O/tail_stamps81.err || exit $?
timeout -k 10 600 $T -v tests/test_gpu_batch.py tests/test_gpu_parity.py > $O/tests_batch.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit $?
P="timeout -s KILL 120 rocprofv3 --kernel-trace --kernel-include-regex cp4d|corr_gemm --output-format csv"
cd /tmp && R=$GRAFT_REPO_ROOT && \
$P --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VALU -d $R/$O/pmc_sq -o run -- python -u $R/tools/time_match.py 1 2 > $R/$O/pmc_sq.log 2>&1 && \
$P --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_WAVES -d $R/$O/pmc_lds -o run -- python -u $R/tools/time_match.py 1 2 > $R/$O/pmc_lds.log 2>&1 && \
$P --pmc FETCH_SIZE -d $R/$O/pmc_fetch -o run -- python -u $R/tools/time_match.py 1 2 > $R/$O/pmc_fetch.log 2>&1 && \
$P --pmc TCC_HIT_sum TCC_MISS_sum -d $R/$O/pmc_tcc -o run -- python -u $R/tools/time_match.py 1 2 > $R/$O/pmc_tcc.log 2>&1 || exit $?
echo done
