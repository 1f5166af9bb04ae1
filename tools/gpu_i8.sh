#!/bin/bash
# int8-digit conv1 in the fp32 torso forward: numerics tests, torso probe, fp32 bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -q -x --timeout 120 --timeout-method thread \
  tests/test_split_gpu.py > gpurun_out/i8_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/i8_tests.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/sp_micro.py torso 20 probe > gpurun_out/i8_probe.json 2>&1 || { tail -5 gpurun_out/i8_probe.json; exit 1; }
head -c 700 gpurun_out/i8_probe.json; echo
timeout -k 10 200 python bench.py --steps 100 > gpurun_out/i8_b1.log 2>&1 || exit 1
grep -h metric gpurun_out/i8_b1.log | cut -c1-60
timeout -k 10 400 python -u -m pytest -q -x --timeout 120 --timeout-method thread \
  tests/test_engine_gpu.py tests/test_actor_gpu.py > gpurun_out/i8_tests2.txt 2>&1
rc=$?; tail -3 gpurun_out/i8_tests2.txt
exit $rc
