# Round-6 A/B: the pipeline's loop at three units per workgroup (40 CUs) against two (59 CUs), with the
# high-priority adapt stream; interleaved, driver's step counts.
set -u
OUT=gpurun_out/r6units
mkdir -p $OUT
for i in 1 2 3; do
  for u in 2 3; do
    CWT_PIPE_ADAPT_UNITS=$u timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --exact-steps 0 --x3-steps 0 --pair-steps 0 > $OUT/bench_u${u}_r$i.json 2> $OUT/bench_u${u}_r$i.err || { echo "bench u$u r$i rc=$?"; exit 1; }
    echo "bench u$u r$i ok"
  done
done
