#!/bin/bash
# rocprofv3 kernel trace of bench.py --force-dp (one rank, RCCL) with / without global sampling:
# where the data-parallel step machinery's overhead goes.  Usage: bash tools/prof_force_dp.sh
set -o pipefail
export TMPDIR=/tmp RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1
mkdir -p gpurun_out
i=0
for gs in 1 0; do
  i=$((i+1))
  export MASTER_PORT=$((29560 + i))
  rm -rf gpurun_out/prof_fdp$gs
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_fdp$gs -- \
    python bench.py --steps 20 --warmup 10 --force-dp --set dist.global_sampling=$gs \
    > gpurun_out/prof_fdp$gs.log 2>&1 || { tail -20 gpurun_out/prof_fdp$gs.log; exit 1; }
  python tools/step_breakdown.py "gpurun_out/prof_fdp$gs/*/*kernel_trace.csv" gpurun_out/fdp$gs.txt 5 > /dev/null
  python tools/step_timeline.py "gpurun_out/prof_fdp$gs/*/*kernel_trace.csv" sample_batch > gpurun_out/fdp${gs}_timeline.txt 2>&1 || true
  head -30 gpurun_out/fdp$gs.txt
  rm -rf gpurun_out/prof_fdp$gs
done
