#!/bin/bash
# Round-3 state of record on one GPU box: smoke + full -m gpu suite + bench (tools/gpu_check.sh),
# then the rocprofv3 kernel-trace stats of the bench command, the PMC passes (tools/pmc.sh)
# and the conv table from the bench's per-launch records.
set -u
TAG=${TAG:-r3}
bash tools/gpu_check.sh && \
OUT=gpurun_out/prof_$TAG STEPS=10 bash tools/profile.sh && \
OUT=gpurun_out/pmc_$TAG bash tools/pmc.sh && \
python tools/pmc_summary.py gpurun_out/pmc_$TAG gpurun_out/pmc_summary_$TAG.json
