#!/bin/bash
# Round-4 state of record, part 2: the driver's bench command, the rocprofv3 kernel stats of the
# SAME command, the PMC passes (separate runs, kernel trace only), the per-conv table, and the
# other operating points (configs #3-#5).
set -u
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=${O:-gpurun_out/r4final}
mkdir -p $O
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --profile-json $O/per_launch.json > $O/bench.json 2> $O/bench.err || exit $?
cd /tmp && R=$GRAFT_REPO_ROOT
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o run -- \
  python -u $R/bench.py --steps 20 --warmup 5 > $R/$O/bench_prof.json 2> $R/$O/bench_prof.err || exit $?
cd $R
OUT=$O/pmc bash tools/pmc.sh > $O/pmc.log 2>&1 || exit $?
python tools/pmc_summary.py $O/pmc $O/pmc_summary.json > /dev/null || exit $?
python tools/conv_table.py $O/per_launch.json > $O/conv_table.md || exit $?
echo done
