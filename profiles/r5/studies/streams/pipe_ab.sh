set -e
mkdir -p gpurun_out/pipe
T="timeout -k 10"
O="--steps 20 --warmup 5 --no-cpu-baseline --exact-steps 0 --x3-steps 0 --pair-steps 0"
for i in 1 2 3; do
$T 300 python -u bench.py $O --pipeline 2 > gpurun_out/pipe/p2_$i.json 2> gpurun_out/pipe/p2_$i.err
$T 300 python -u bench.py $O --pipeline 3 > gpurun_out/pipe/p3_$i.json 2> gpurun_out/pipe/p3_$i.err
done
