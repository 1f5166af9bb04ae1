set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -q -x --timeout 120 --timeout-method thread tests/test_gemm_sp_gpu.py > gpurun_out/g5_tests.txt 2>&1 || { tail -20 gpurun_out/g5_tests.txt; exit 1; }
tail -1 gpurun_out/g5_tests.txt
timeout -k 10 200 python tools/gemm_sp_micro.py > gpurun_out/g5_micro.json 2>gpurun_out/g5_micro.err || { tail -5 gpurun_out/g5_micro.err; exit 1; }
cat gpurun_out/g5_micro.json
timeout -k 10 200 python bench.py --steps 200 > gpurun_out/g5_bench.log 2>&1 || exit 1
grep -h metric gpurun_out/g5_bench.log | cut -c1-60
