set -e
mkdir -p gpurun_out/knobs
T="timeout -k 10"
O="--steps 20 --warmup 5 --no-cpu-baseline --exact-steps 0 --x3-steps 0 --pair-steps 0"
for i in 1 2 3 4; do
$T 300 python -u bench.py $O > gpurun_out/knobs/base_$i.json 2> gpurun_out/knobs/base_$i.err
CWT_ADAPT_PR=4 $T 300 python -u bench.py $O > gpurun_out/knobs/pr4_$i.json 2> gpurun_out/knobs/pr4_$i.err
CWT_ADAPT_PR=16 $T 300 python -u bench.py $O > gpurun_out/knobs/pr16_$i.json 2> gpurun_out/knobs/pr16_$i.err
CWT_PIPE_DRAIN_OVERLAP=1 $T 300 python -u bench.py $O > gpurun_out/knobs/dov_$i.json 2> gpurun_out/knobs/dov_$i.err
done
