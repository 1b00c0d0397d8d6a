# Round-6 configs #3-#5 (BASELINE.json configs), one bench line each, builder-timed.
set -u
OUT=gpurun_out/r6cfg
mkdir -p $OUT
timeout -k 10 600 python -u bench.py --shot 5 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/c3.json 2> $OUT/c3.err || { echo "c3 rc=$?"; exit 1; }
timeout -k 10 600 python -u bench.py --train --layers 101 --size 641 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/c4.json 2> $OUT/c4.err || { echo "c4 rc=$?"; exit 1; }
timeout -k 10 600 python -u bench.py --shot 5 --layers 101 --size 641 --conv-dtype bf16 --steps 20 --warmup 5 --no-cpu-baseline --profile-json $OUT/c5_prof.json > $OUT/c5.json 2> $OUT/c5.err || { echo "c5 rc=$?"; exit 1; }
echo "configs ok"
timeout -k 10 900 python -u tools/conv_s_sweep.py --prec 1 --configs 101:641:6 --vars 0,1,2,4 --reps 10 --out r6cfg/sweep_b16_101_641_6.json > $OUT/sweep_b16.log 2>&1
echo "b16 sweep rc=$?"
