set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -q -x --timeout 120 --timeout-method thread tests/test_split_gpu.py > gpurun_out/tb_tests.txt 2>&1 || { tail -20 gpurun_out/tb_tests.txt; exit 1; }
tail -1 gpurun_out/tb_tests.txt
timeout -k 10 120 python tools/torso_bwd_sp_probe.py > gpurun_out/tb_probe.json 2>gpurun_out/tb_probe.err || { tail -5 gpurun_out/tb_probe.err; exit 1; }
tail -c 900 gpurun_out/tb_probe.json
timeout -k 10 200 python bench.py --steps 200 > gpurun_out/tb_bench.log 2>&1 || exit 1
grep -h metric gpurun_out/tb_bench.log | cut -c1-60
