#!/bin/bash
# Same-box per-kernel comparison of two trees' bench step (rocprofv3 kernel traces):
#   tools/prof_pair.sh name=dir[:bench args] ...   -> gpurun_out/pp_<name>/..., medians printed
set -o pipefail
export TMPDIR=/tmp
root=$(pwd)
for spec in "$@"; do
  name=${spec%%=*}; rest=${spec#*=}; dir=${rest%%:*}; args=""
  [[ "$rest" == *:* ]] && args=${rest#*:}
  rm -rf "$root/gpurun_out/pp_$name"
  (cd "$dir" && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$root/gpurun_out/pp_$name" -- \
     python bench.py --steps 20 --warmup 10 $args > "$root/gpurun_out/pp_$name.log" 2>&1) || { echo "FAIL $name"; tail -5 "$root/gpurun_out/pp_$name.log"; exit 1; }
  echo "== $name ($dir $args) $(grep -o '"ms_per_step": [0-9.]*' "$root/gpurun_out/pp_$name.log")"
  python "$root/tools/kernel_medians.py" "$root/gpurun_out/pp_$name/*/*kernel_trace.csv" torso lstm gemm6 td_duel prio_tail rmsprop pack_step sample
done
