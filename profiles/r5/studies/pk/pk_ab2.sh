set -e
mkdir -p gpurun_out/pk2
T="timeout -k 10"
for i in 1 2; do
CWT_LIB_PATH=tools/ab/libpk0.so $T 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/pk2/bench_pk0_$i.json 2> gpurun_out/pk2/bench_pk0_$i.err
$T 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/pk2/bench_pk1_$i.json 2> gpurun_out/pk2/bench_pk1_$i.err
done
