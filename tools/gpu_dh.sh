#!/bin/bash
# Validate the fused TD dh path: GPU tests touching it, then fp32/bf16 benches and an A/B with it off.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -q -x --timeout 120 --timeout-method thread \
  tests/test_split_gpu.py tests/test_engine_gpu.py tests/test_actor_gpu.py > gpurun_out/dh_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/dh_tests.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --steps 100 > gpurun_out/b1.log 2>&1 &&
timeout -k 10 200 python bench.py --dtype bf16 --steps 100 > gpurun_out/b2.log 2>&1 &&
timeout -k 10 200 python bench.py --steps 100 --set learner.td_fuse_dh=false > gpurun_out/b3.log 2>&1
rc=$?
grep -h metric gpurun_out/b1.log gpurun_out/b2.log gpurun_out/b3.log | cut -c1-110
exit $rc
