set -o pipefail
mkdir -p gpurun_out
for env in "X=1" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=0" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=1" "ROC_SYSTEM_SCOPE_SIGNAL=0" "DEBUG_HIP_GRAPH_BATCH_SIZE=64" "HIP_FORCE_DEV_KERNARG=1" "GPU_FLUSH_ON_EXECUTION=0"; do
  r=$(env $env timeout -k 10 120 python bench.py --steps 300 --warmup 30 2>/dev/null | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])") || { echo "$env FAILED"; exit 1; }
  echo "$env $r"
done
