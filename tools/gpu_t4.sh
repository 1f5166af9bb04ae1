set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python tools/lstm_sp_probe.py > gpurun_out/lstm_t4_probe.json 2>gpurun_out/lstm_t4_probe.err || { tail -5 gpurun_out/lstm_t4_probe.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/lstm_t4_probe.json')); print({k: v for k, v in d.items() if 'trace_poll' not in k})"
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_split_gpu.py tests/test_engine_gpu.py > gpurun_out/pytest_t4.txt 2>&1 || { tail -30 gpurun_out/pytest_t4.txt; exit 1; }
tail -1 gpurun_out/pytest_t4.txt
timeout -k 10 200 python bench.py --steps 200 > gpurun_out/bench_t4.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --steps 200 --target-mode reference > gpurun_out/bench_t4_ref.log 2>&1 || exit 1
grep -h metric gpurun_out/bench_t4.log gpurun_out/bench_t4_ref.log | cut -c1-100
