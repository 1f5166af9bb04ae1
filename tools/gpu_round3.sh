set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
echo SMOKE ok
timeout -k 10 700 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/pytest_gpu.txt 2>&1 || { tail -30 gpurun_out/pytest_gpu.txt; exit 1; }
tail -1 gpurun_out/pytest_gpu.txt
timeout -k 10 200 python bench.py > gpurun_out/bench_default.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --steps 200 > gpurun_out/bench_fp32_200.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --dtype bf16 --steps 200 > gpurun_out/bench_bf16.log 2>&1 || exit 1
grep -h metric gpurun_out/bench_default.log gpurun_out/bench_fp32_200.log gpurun_out/bench_bf16.log | cut -c1-110
bash tools/prof_bench.sh fp32_r3 || exit 1
