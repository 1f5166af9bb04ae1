#!/bin/bash
# bench.py under several config-override sets, one line each.  Each argument is a
# space-separated list of KEY=VALUE overrides ("" = defaults).
for v in "$@"; do
  sets=""; for kv in $v; do sets="$sets --set $kv"; done
  timeout -k 10 150 python bench.py --steps 300 --warmup 30 $sets > gpurun_out/bs.log 2>&1 || { echo "FAIL [$v]"; tail -5 gpurun_out/bs.log; exit 1; }
  echo "[$v] $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bs.log)"
done
