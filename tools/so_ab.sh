#!/bin/bash
# Same-box A/B of kernel-library builds (run through gpurun from the repo root):
#   tools/so_ab.sh ROUNDS name=path/to/_r2d2_kernels.so ...    (extra bench.py args: $BENCH_ARGS)
# Each round runs bench.py once per build (interleaved), swapping the in-tree library between
# processes; the original library is restored at the end or on the first failure.
set -o pipefail
mkdir -p gpurun_out
so=pytorch_r2d2_amd/_r2d2_kernels.so
cp "$so" gpurun_out/.so_orig
rounds=$1; shift
for r in $(seq 1 "$rounds"); do
  for spec in "$@"; do
    name=${spec%%=*}; path=${spec#*=}
    cp "$path" "$so"
    if ! timeout -k 10 180 python bench.py --steps 300 --warmup 30 $BENCH_ARGS > gpurun_out/so_ab.log 2>&1; then
      cp gpurun_out/.so_orig "$so"; echo "FAIL $name"; tail -20 gpurun_out/so_ab.log; exit 1
    fi
    echo "$name $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/so_ab.log)"
  done
done
cp gpurun_out/.so_orig "$so"
