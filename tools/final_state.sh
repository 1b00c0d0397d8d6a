set -u
bash tools/gpu_check.sh || exit $?
OUT=gpurun_out/prof_final STEPS=10 bash tools/profile.sh || exit $?
OUT=gpurun_out/prof_final_bf16 STEPS=10 BENCH_ARGS="--conv-dtype bf16" bash tools/profile.sh || exit $?
OUT=gpurun_out/pmc_final bash tools/pmc.sh || exit $?
OUT=gpurun_out/pmc_final_bf16 BENCH_ARGS="--conv-dtype bf16" bash tools/pmc.sh || exit $?
