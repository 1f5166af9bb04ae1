#!/bin/bash
# bench.py under several R2D2_BWD_GEMM settings (one line each)
for v in "$@"; do
  R2D2_BWD_GEMM="$v" timeout -k 10 120 python bench.py --steps 300 --warmup 30 > gpurun_out/bg.log 2>&1 || { echo "FAIL $v"; tail -5 gpurun_out/bg.log; exit 1; }
  echo "bwd_gemm=[$v] $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bg.log)"
done
