#!/bin/bash
# rocprofv3 kernel trace of a short bench run with extra bench args + step breakdown
# usage: tools/prof_cfg.sh <tag> [bench args...]
export TMPDIR=/tmp
tag=$1; shift
rm -rf gpurun_out/prof_$tag
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$tag -- python bench.py --steps 20 --warmup 10 "$@" > gpurun_out/prof_$tag.log 2>&1 || { echo "PROF FAIL $tag"; tail -5 gpurun_out/prof_$tag.log; exit 1; }
grep metric gpurun_out/prof_$tag.log | cut -c1-120
python tools/step_breakdown.py "gpurun_out/prof_$tag/*/*kernel_trace.csv" gpurun_out/$tag.txt 5 > /dev/null
head -40 gpurun_out/$tag.txt
