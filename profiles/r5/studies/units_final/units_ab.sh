set -e
mkdir -p gpurun_out/units
T="timeout -k 10"
O="--steps 20 --warmup 5 --no-cpu-baseline --exact-steps 0 --x3-steps 0 --pair-steps 0"
for i in 1 2 3 4; do
for u in 2 3 1; do
CWT_PIPE_ADAPT_UNITS=$u $T 300 python -u bench.py $O > gpurun_out/units/u${u}_$i.json 2> gpurun_out/units/u${u}_$i.err
done
CWT_PIPE_ADAPT_PRIO=1 $T 300 python -u bench.py $O > gpurun_out/units/prio_$i.json 2> gpurun_out/units/prio_$i.err
done
