set -e
mkdir -p gpurun_out/dvfs
O="--warmup 5 --no-cpu-baseline --exact-steps 0 --x3-steps 0 --pair-steps 0"
timeout -k 5 20 amd-smi metric -g 0 -c > gpurun_out/dvfs/idle.txt 2>&1 || true
(for i in $(seq 1 60); do date +%s.%N; timeout -k 2 5 amd-smi metric -g 0 -c -p 2>&1 || true; sleep 0.05; done) > gpurun_out/dvfs/smi_pipe.txt 2>&1 &
SP=$!
timeout -k 10 300 python -u bench.py --steps 1500 $O > gpurun_out/dvfs/bench_1500.json 2> gpurun_out/dvfs/bench_1500.err
kill $SP 2>/dev/null || true
wait $SP 2>/dev/null || true
(for i in $(seq 1 40); do date +%s.%N; timeout -k 2 5 amd-smi metric -g 0 -c -p 2>&1 || true; sleep 0.05; done) > gpurun_out/dvfs/smi_loop.txt 2>&1 &
SP=$!
CWT_ADAPT_UPW=2 timeout -k 10 200 python -u tools/time_adapt.py 1 473 3000 > gpurun_out/dvfs/loop.json 2> gpurun_out/dvfs/loop.err
kill $SP 2>/dev/null || true
wait $SP 2>/dev/null || true
