set -u
mkdir -p gpurun_out
for R in 4 8 16 32; do
  CWT_ADAPT_R=$R SHOTS=1 FLAGS=0 timeout -k 10 120 python -u tools/adapt_ablate.py > gpurun_out/abl_R$R.log 2>&1 || exit $?
  echo "R=$R $(tail -1 gpurun_out/abl_R$R.log)"
done
