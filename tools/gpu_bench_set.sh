#!/bin/bash
# Several bench.py lines in one GPU call: BENCH_SETS="name1|args1;name2|args2"; stops on crash.
mkdir -p gpurun_out
stop_if_crash() { case $1 in 124|134|137|139) echo "CRASH rc=$1 -> stopping"; exit $1;; esac; }
IFS=';' read -ra SETS <<< "$BENCH_SETS"
for s in "${SETS[@]}"; do
  name="${s%%|*}"; args="${s#*|}"
  timeout -k 10 ${BENCH_TIMEOUT:-300} python bench.py $args > "gpurun_out/bench_$name.log" 2>&1; rc=$?
  echo "BENCH $name rc=$rc: $(grep -o '"value": [0-9.]*' gpurun_out/bench_$name.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_$name.log)"
  stop_if_crash $rc
done
exit 0
