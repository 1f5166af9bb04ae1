#!/bin/bash
# bench.py under several R2D2_BPTT_HELPERS settings (one line each)
for v in "$@"; do
  R2D2_BPTT_HELPERS="$v" timeout -k 10 120 python bench.py --steps 200 --warmup 20 > gpurun_out/bv.log 2>&1 || { echo "FAIL $v"; tail -5 gpurun_out/bv.log; exit 1; }
  echo "helpers=[$v] $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bv.log)"
done
