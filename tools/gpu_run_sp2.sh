set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_split_gpu.py tests/test_engine_gpu.py > gpurun_out/split_tests.txt 2>&1 || { tail -30 gpurun_out/split_tests.txt; exit 1; }
tail -3 gpurun_out/split_tests.txt
timeout -k 10 200 python bench.py --steps 100 --warmup 10 > gpurun_out/bench_fp32.log 2>&1 || exit 1
grep metric gpurun_out/bench_fp32.log | cut -c1-300
bash tools/prof_bench.sh fp32_v2
timeout -k 10 200 python bench.py --steps 100 --warmup 10 --dtype bf16 > gpurun_out/bench_bf16.log 2>&1 || exit 1
grep metric gpurun_out/bench_bf16.log | cut -c1-200
