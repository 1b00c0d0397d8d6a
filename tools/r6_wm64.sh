# Round-6 study: x6 forms with WM = 64 rows per wave (var 6: 128x128 in 2x1 waves; var 7: 256x128 in
# 4x1 waves; one wave per SIMD, B fragments reused over 4 A fragments) against var 5, layer3/4 + the
# Winograd GEMMs at 1-shot 473.
set -u
OUT=gpurun_out/r6wm64
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv_s.py -m gpu -x -q --timeout 120 --timeout-method thread -k "x6_plans" > $OUT/pytest.txt 2>&1 || { echo "pytest rc=$?"; exit 1; }
echo "pytest ok"
timeout -k 10 600 python -u tools/conv_s_sweep.py --prec 6 --configs 50:473:2 --vars 5,6,7 --only l3c1,l3down,l3c3,l4c1,l4down,l4c3 --reps 10 --out r6wm64/p6.json > $OUT/p6.log 2>&1 || { echo "p6 rc=$?"; exit 1; }
echo "p6 ok"
timeout -k 10 600 python -u tools/conv_s_sweep.py --prec 7 --configs 50:473:2 --vars 5,6,7 --only l3c2,l4c2,bottleneck --reps 10 --out r6wm64/p7.json > $OUT/p7.log 2>&1 || { echo "p7 rc=$?"; exit 1; }
echo "p7 ok"
