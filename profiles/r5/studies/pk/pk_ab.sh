set -e
mkdir -p gpurun_out/pk
T="timeout -k 10"
$T 600 python -u -m pytest tests/test_gpu_adapt_persist.py tests/test_gpu_tail.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "persist or fused or inner_loop or tail or step" > gpurun_out/pk/tests.log 2>&1
for i in 1 2 3; do
  CWT_ADAPT_UPW=2 $T 120 python -u tools/time_adapt.py 1 473 60 >> gpurun_out/pk/time_adapt.jsonl
  CWT_ADAPT_UPW=2 CWT_LIB_PATH=tools/ab/libpk0.so $T 120 python -u tools/time_adapt.py 1 473 60 >> gpurun_out/pk/time_adapt.jsonl
done
$T 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/pk/bench_pk1.json 2> gpurun_out/pk/bench_pk1.err
CWT_LIB_PATH=tools/ab/libpk0.so $T 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/pk/bench_pk0.json 2> gpurun_out/pk/bench_pk0.err
