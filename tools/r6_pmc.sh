# Round-6 state of record, part 2: the PMC passes (tools/pmc.sh: FETCH_SIZE, WRITE_SIZE, SQ, LDS,
# each its own rocprofv3 run) over a short bench run.
set -u
OUT=gpurun_out/r6p bash tools/pmc.sh
