set -u
mkdir -p gpurun_out/r6e
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --profile-json gpurun_out/r6e/prof.json > gpurun_out/r6e/bench.json 2> gpurun_out/r6e/bench.err || exit $?
timeout -k 10 400 python -u tools/conv_s_sweep.py --prec 6 --vars 5,6 --reps 20 --only l3c3,l3c1,l3down,l4c1,l4c3,l4down --out r6e/sweep_v6.json > gpurun_out/r6e/sweep_v6.log 2>&1 || exit $?
timeout -k 10 400 python -u tools/conv_s_sweep.py --prec 7 --vars 5,6 --reps 10 --out r6e/sweep_p7_v6.json > gpurun_out/r6e/sweep_p7_v6.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/x6_decomp.py --vars 5,17,18 --only l2c3,l3c3,l4c3 --out r6e/x6_launch.json > gpurun_out/r6e/x6_launch.log 2>&1 || exit $?
timeout -k 10 900 python -u tools/conv_s_sweep.py --prec 6 --configs 50:473:6,101:641:2 --vars 0,1,2,3,4,5 --reps 10 --only stem2,stem3,l1c1,l1c2,l1c3,l1down,l2c1,l2c2,l2c3,l2down --out r6e/sweep_small_c34.json > gpurun_out/r6e/sweep_small_c34.log 2>&1
echo rc=$?
