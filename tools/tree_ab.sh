#!/bin/bash
# Same-box A/B of whole source trees / knob settings (run through gpurun from the repo root):
#   tools/tree_ab.sh ROUNDS name=dir[:bench args] ...   (dir: a tree with its own built libraries;
#   "." = this one).  Each round runs each arm's bench.py once (interleaved), 300 timed steps;
#   extra bench args for every arm: $BENCH_ARGS.
set -o pipefail
mkdir -p gpurun_out
rounds=$1; shift
for r in $(seq 1 "$rounds"); do
  for spec in "$@"; do
    name=${spec%%=*}; rest=${spec#*=}; dir=${rest%%:*}; args=""
    [[ "$rest" == *:* ]] && args=${rest#*:}
    if ! (cd "$dir" && timeout -k 10 180 python bench.py --steps 300 --warmup 30 $args $BENCH_ARGS) > gpurun_out/tree_ab.log 2>&1; then
      echo "FAIL $name"; tail -20 gpurun_out/tree_ab.log; exit 1
    fi
    echo "$name $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/tree_ab.log)"
  done
done
