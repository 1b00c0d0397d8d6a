# Round-6 A/B: a high-priority adapt stream (CWT_PIPE_ADAPT_PRIO=1) against the default, interleaved:
# does the loop's grid get its CUs sooner (its pipelined launch time), and does the rate move?
set -u
OUT=gpurun_out/r6prio
mkdir -p $OUT
for i in ${ROUNDS:-1 2 3}; do
  for pr in 0 1; do
    CWT_PIPE_ADAPT_PRIO=$pr timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --exact-steps 0 --x3-steps 0 --pair-steps 0 > $OUT/bench_prio${pr}_r$i.json 2> $OUT/bench_prio${pr}_r$i.err || { echo "bench prio$pr r$i rc=$?"; exit 1; }
    echo "bench prio$pr r$i ok"
  done
done
