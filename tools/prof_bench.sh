#!/bin/bash
# rocprofv3 kernel trace of a short bench run + per-step kernel breakdown -> gpurun_out/$1.txt
# usage: tools/prof_bench.sh <tag>   (env vars pass through to bench.py)
export TMPDIR=/tmp
rm -rf gpurun_out/prof_$1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$1 -- python bench.py --steps 20 --warmup 10 > gpurun_out/prof_$1.log 2>&1 || { echo "PROF FAIL $1"; tail -5 gpurun_out/prof_$1.log; exit 1; }
python tools/step_breakdown.py "gpurun_out/prof_$1/*/*kernel_trace.csv" gpurun_out/$1.txt 5 > /dev/null
head -14 gpurun_out/$1.txt
