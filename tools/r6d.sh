set -u
mkdir -p gpurun_out/r6d
timeout -k 10 300 python -u tools/x6_decomp.py --out r6d/x6_decomp_rpf.json > gpurun_out/r6d/decomp_rpf.log 2>&1 || exit $?
timeout -k 10 800 python -u tools/conv_s_sweep.py --prec 6 --vars 0,1,2,3,4,5 --reps 20 --only stem2,stem3,l1c1,l1c2,l1c3,l1down,l2c1,l2c2,l2c3,l2down --out r6d/sweep_small.json > gpurun_out/r6d/sweep_small.log 2>&1
echo rc=$?
