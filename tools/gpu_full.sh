set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/pytest_gpu.txt 2>&1 || { tail -30 gpurun_out/pytest_gpu.txt; exit 1; }
tail -2 gpurun_out/pytest_gpu.txt
bash tools/prof_cfg.sh dm3 --config dmlab30 || exit 1
timeout -k 10 200 python bench.py --steps 100 --warmup 10 > gpurun_out/bench_fp32.log 2>&1 || exit 1
grep metric gpurun_out/bench_fp32.log | cut -c1-150
