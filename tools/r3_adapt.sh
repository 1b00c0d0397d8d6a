#!/bin/bash
# round-3 inner-loop check: persist-vs-step parity (incl. the three-unit lockstep form), then
# A/B timing of the loop alone against the previous build (tools/ab/lib_old.so)
set -o pipefail
O=${1:-gpurun_out/r3h}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -v -x --timeout 120 --timeout-method thread tests/test_gpu_adapt_persist.py > $O/persist_tests.log 2>&1 || exit 1
for cfg in "1 473" "5 473" "5 641" "1 641"; do
  for lib in tools/ab/lib_old.so few_shot_seg_cwt_amd/libcwt.so; do
    CWT_LIB_PATH=$lib timeout -k 10 120 python -u tools/time_adapt.py $cfg 30 >> $O/time_adapt.jsonl 2>> $O/time_adapt.err || exit 1
  done
done
for lib in tools/ab/lib_old.so few_shot_seg_cwt_amd/libcwt.so; do
  CWT_ADAPT_UPW=2 CWT_LIB_PATH=$lib timeout -k 10 120 python -u tools/time_adapt.py 1 473 30 >> $O/time_adapt.jsonl 2>> $O/time_adapt.err || exit 1
done
