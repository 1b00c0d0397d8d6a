# Round-6 study: the layer1-3 conv plans timed while 59 CUs are held (the pipeline's resident inner
# loop overlaps those layers), beside the same sweep with every CU free.
set -u
OUT=gpurun_out/r6occ
mkdir -p $OUT
SH=l1c1,l1c2,l1c3,l1down,l2c1,l2c2,l2down,l2c3,l3c1,l3down,l3c3
timeout -k 10 600 python -u tools/conv_s_sweep.py --prec 6 --configs 50:473:2 --vars 0,1,2,3,4,5 --only $SH --reps 10 --occupy 59 --out r6occ/occ59_p6.json > $OUT/occ59_p6.log 2>&1 || { echo "occ59 p6 rc=$?"; exit 1; }
echo "occ59 p6 ok"
timeout -k 10 300 python -u tools/conv_s_sweep.py --prec 7 --configs 50:473:2 --vars 0,1,2,3,4,5 --only l3c2 --reps 10 --occupy 59 --out r6occ/occ59_p7.json > $OUT/occ59_p7.log 2>&1 || { echo "occ59 p7 rc=$?"; exit 1; }
echo "occ59 p7 ok"
echo "solo p6 skipped"
echo "solo p6 ok"
echo "solo p7 skipped"
echo "solo p7 ok"
