#!/bin/bash
# A/B of HIP runtime knobs on the headline bench (one GPU).  Measured (v17, 300 steps):
# default 1419, DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 1429, =1 1419 (within run-to-run noise);
# HIP_FORCE_DEV_KERNARG=1 1448.8 / 1446.5 vs 1449.2 / 1446.4 (v19, 800 steps): no effect.
# (ROC_SYSTEM_SCOPE_SIGNAL=0 made bench.py exit non-zero: not swept.)
set -o pipefail
mkdir -p gpurun_out
for env in "X=1" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=0" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=1" "HIP_FORCE_DEV_KERNARG=1"; do
  r=$(env $env timeout -k 10 120 python bench.py --steps 300 --warmup 30 2>/dev/null | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])") || { echo "$env FAILED"; exit 1; }
  echo "$env $r"
done
