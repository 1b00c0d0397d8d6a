#!/bin/bash
# Round 4, box x: where the rolling-window consensus kernels' time goes -- the layer timings with
# the loads or the arithmetic skipped (CWT_CP4D_RDBG 2 / 1 / 3), and PMC passes over the layer
# timing tool (SQ busy / wait / LDS, HBM fetch and write).
set -u
export TMPDIR=/tmp PYTHONUNBUFFERED=1
R=$(pwd)
O=gpurun_out/r4x
mkdir -p $O
for d in 0 1 2 3; do
  CWT_CP4D_RDBG=$d timeout -k 10 120 python -u tools/time_cp4d.py 10 | sed "s/^{/{\"rdbg\": $d, /" >> $O/time_cp4d.jsonl 2>> $O/time.err || exit $?
done
P="timeout -s KILL 120 rocprofv3"
$P --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VALU -d $R/$O/pmc_sq -o run -- python3 -u $R/tools/time_cp4d.py 2 > $R/$O/pmc_sq.log 2>&1 && \
$P --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_WAVES -d $R/$O/pmc_lds -o run -- python3 -u $R/tools/time_cp4d.py 2 > $R/$O/pmc_lds.log 2>&1 && \
$P --pmc FETCH_SIZE -d $R/$O/pmc_fetch -o run -- python3 -u $R/tools/time_cp4d.py 2 > $R/$O/pmc_fetch.log 2>&1 && \
$P --pmc WRITE_SIZE -d $R/$O/pmc_write -o run -- python3 -u $R/tools/time_cp4d.py 2 > $R/$O/pmc_write.log 2>&1 || exit $?
echo done
