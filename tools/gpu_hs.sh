set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_split_gpu.py tests/test_kernels_gpu.py tests/test_engine_gpu.py > gpurun_out/hs_tests.txt 2>&1 || { tail -30 gpurun_out/hs_tests.txt; exit 1; }
tail -1 gpurun_out/hs_tests.txt
timeout -k 10 120 python tools/lstm_sp_probe.py > gpurun_out/hs_probe.json 2>gpurun_out/hs_probe.err || { tail -5 gpurun_out/hs_probe.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/hs_probe.json').read().strip().split('\n')[-1]); print({k: v for k, v in d.items() if 'trace_poll' not in k})"
timeout -k 10 200 python bench.py --steps 300 > gpurun_out/hs_b.log 2>&1 || exit 1
grep -h metric gpurun_out/hs_b.log | cut -c1-60
timeout -k 10 200 python bench.py --steps 300 --dtype bf16 > gpurun_out/hs_bf.log 2>&1 || exit 1
grep -h metric gpurun_out/hs_bf.log | cut -c1-60
