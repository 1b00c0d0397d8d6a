#!/bin/bash
# Round 4, box h: persistent CenterPivotConv4d timing study -- kernel stats with the staging
# only (CWT_CP4D_DBG=1), the compute only (2), both (default) and the tile kernels.
set -u
export TMPDIR=/tmp
O=gpurun_out/r4h
mkdir -p $O
cd /tmp && R=$GRAFT_REPO_ROOT
for v in def dbg1 dbg2 tile; do
  case $v in
    def) E="" ;; dbg1) E="CWT_CP4D_DBG=1" ;; dbg2) E="CWT_CP4D_DBG=2" ;; tile) E="CWT_CP4D_PERSIST=0" ;;
  esac
  export CWT_CP4D_DBG=0 CWT_CP4D_PERSIST=1
  [ -n "$E" ] && export $E
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_$v -o run -- \
    python -u $R/tools/time_match.py 1 3 > $R/$O/time_$v.json 2> $R/$O/time_$v.err || exit $?
done
echo done
