# Round-6 state of record, part 1 (one GPU session): smoke, the driver's bench command, the same
# command under rocprofv3 --kernel-trace --stats.  Every GPU step under its own time limit; a
# failure ends the script.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r6s
mkdir -p $OUT
timeout -k 10 300 python -u __graft_entry__.py smoke > $OUT/smoke.log 2>&1 || { echo "smoke rc=$?"; exit 1; }
echo "smoke ok"
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 --profile-json $OUT/prof.json > $OUT/bench.json 2> $OUT/bench.err || { echo "bench rc=$?"; exit 1; }
echo "bench ok"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/rocprof -o run -- \
  python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/prof_bench.json 2> $OUT/prof_bench.err || { echo "rocprof rc=$?"; exit 1; }
echo "rocprof ok"
