#!/bin/bash
# PMC counter passes over a short bench run, one rocprofv3 process per pass (kernel-trace only,
# no sys/runtime traces): HBM bytes (FETCH_SIZE, WRITE_SIZE: separate passes, they do not fit
# one TCC pass) and an SQ pass for MFMA busy / stall breakdown.  Output: $OUT/<pass>/...
set -u
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/pmc_r1}
mkdir -p $OUT
run_pass() {
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc "$@" --output-format csv -d $OUT/$name -o run -- \
    python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --exact-steps 2 --x3-steps 2 --pair-steps 0 ${BENCH_ARGS:-} > $OUT/$name.bench.json 2> $OUT/$name.err
  local rc=$?
  echo "pass $name rc=$rc"
  return $rc
}
run_pass fetch FETCH_SIZE && \
run_pass write WRITE_SIZE && \
run_pass sq SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VALU GRBM_GUI_ACTIVE && \
run_pass lds SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES
