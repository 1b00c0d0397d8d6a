# Round-6 repeats of the driver's default bench command on the final code (run-to-run spread).
set -u
OUT=gpurun_out/r6rep
mkdir -p $OUT
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $OUT/bench_$i.json 2> $OUT/bench_$i.err || { echo "bench $i rc=$?"; exit 1; }
  echo "bench $i ok"
done
