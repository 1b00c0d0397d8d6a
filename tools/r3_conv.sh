#!/bin/bash
# round-3 conv check: per-conv parity of every plan, then plan sweeps (x3s and bf16) per config
set -o pipefail
O=gpurun_out/r3g
mkdir -p $O
timeout -k 10 300 python -u -m pytest -q -x --timeout 120 --timeout-method thread tests/test_gpu_conv_s.py tests/test_gpu_conv.py > $O/tests.log 2>&1 || exit 1
for prec in 3 1; do
  for c in 50:473:2 50:473:6 101:641:2 101:641:6 50:473:8; do
    timeout -k 10 200 python -u tools/conv_s_sweep.py --prec $prec --configs $c --out r3g/p${prec}_$c.json > $O/p${prec}_$c.log 2>&1 || exit 1
  done
done
