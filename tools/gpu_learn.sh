set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/learn_check.py --steps 3000 --dtype both > gpurun_out/learn.txt 2>gpurun_out/learn.err || { tail -5 gpurun_out/learn.err; exit 1; }
cat gpurun_out/learn.txt
timeout -k 10 300 python bench.py --steps 5000 --warmup 20 > gpurun_out/bench_long.log 2>&1 || { tail -5 gpurun_out/bench_long.log; exit 1; }
grep -h metric gpurun_out/bench_long.log | cut -c1-100
