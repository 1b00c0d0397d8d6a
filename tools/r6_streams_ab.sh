# Round-6 A/B: one extractor stream against the default two, interleaved (driver's step counts).
set -u
OUT=gpurun_out/r6streams
mkdir -p $OUT
for i in 1 2 3; do
  for ps in 2 1; do
    timeout -k 10 300 python -u bench.py --pipeline $ps --steps 20 --warmup 5 --no-cpu-baseline --exact-steps 0 --x3-steps 0 --pair-steps 0 > $OUT/bench_p${ps}_r$i.json 2> $OUT/bench_p${ps}_r$i.err || { echo "bench p$ps r$i rc=$?"; exit 1; }
    echo "bench p$ps r$i ok"
  done
done
