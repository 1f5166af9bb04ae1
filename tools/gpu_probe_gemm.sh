#!/bin/bash
# gemm_sp bound probe + a kernel-trace step breakdown of the default fp32 bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 180 python tools/gemm_sp_bound_probe.py > gpurun_out/gemm_bound.json 2>&1 || { tail -20 gpurun_out/gemm_bound.json; exit 1; }
cat gpurun_out/gemm_bound.json
bash tools/prof_cfg.sh fp32_dh
