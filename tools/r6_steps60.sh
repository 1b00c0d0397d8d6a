# Round-6: the default bench at 60 timed steps (the burst's fill and drain weigh a third as much)
set -u
OUT=gpurun_out/r6s60
mkdir -p $OUT
timeout -k 10 400 python -u bench.py --steps 60 --warmup 5 --no-cpu-baseline --exact-steps 0 --x3-steps 0 --pair-steps 0 > $OUT/bench60.json 2> $OUT/bench60.err || { echo "bench60 rc=$?"; exit 1; }
echo "bench60 ok"
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --exact-steps 0 --x3-steps 0 --pair-steps 0 > $OUT/bench20.json 2> $OUT/bench20.err || { echo "bench20 rc=$?"; exit 1; }
echo "bench20 ok"
