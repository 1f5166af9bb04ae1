#!/bin/bash
# two-groups-per-XCD LSTM forward placement: tests, then benches A/B (fp32 / bf16)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -q -x --timeout 120 --timeout-method thread \
  tests/test_kernels_gpu.py -k "lstm" > gpurun_out/map2_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/map2_tests.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest -q -x --timeout 120 --timeout-method thread \
  tests/test_split_gpu.py tests/test_engine_gpu.py > gpurun_out/map2_tests2.txt 2>&1
rc=$?; tail -3 gpurun_out/map2_tests2.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --steps 100 > gpurun_out/m1.log 2>&1 &&
timeout -k 10 200 python bench.py --steps 100 --set learner.lstm_xcd_pairs=false > gpurun_out/m2.log 2>&1 &&
timeout -k 10 200 python bench.py --dtype bf16 --steps 100 > gpurun_out/m3.log 2>&1 &&
timeout -k 10 200 python bench.py --dtype bf16 --steps 100 --set learner.lstm_xcd_pairs=false > gpurun_out/m4.log 2>&1
rc=$?
grep -h metric gpurun_out/m1.log gpurun_out/m2.log gpurun_out/m3.log gpurun_out/m4.log | cut -c1-60
exit $rc
