#!/bin/bash
# One GPU round-trip: build, smoke, GPU tests, short bench.  Stops after any crash/timeout.
mkdir -p gpurun_out
stop_if_crash() { case $1 in 124|134|137|139) echo "CRASH rc=$1 -> stopping"; exit $1;; esac; }
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { cat gpurun_out/build.log; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
echo "SMOKE rc=$rc"; tail -5 gpurun_out/smoke.log; stop_if_crash $rc
timeout -k 10 ${PYTEST_TIMEOUT:-900} python -m pytest tests -m gpu -q ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "PYTEST rc=$rc"; tail -40 gpurun_out/pytest_gpu.log; stop_if_crash $rc
if [ -n "$BENCH_ARGS" ]; then
  timeout -k 10 ${BENCH_TIMEOUT:-600} python bench.py $BENCH_ARGS > gpurun_out/bench.log 2>&1; rc=$?
  echo "BENCH rc=$rc"; tail -15 gpurun_out/bench.log; stop_if_crash $rc
fi
if [ -n "$PROF_ARGS" ]; then
  export TMPDIR=/tmp
  rm -rf gpurun_out/prof
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -- python bench.py $PROF_ARGS > gpurun_out/prof.log 2>&1; rc=$?
  echo "PROF rc=$rc"; grep metric gpurun_out/prof.log | tail -1; stop_if_crash $rc
  python tools/step_breakdown.py "gpurun_out/prof/*/*kernel_trace.csv" gpurun_out/breakdown.txt 5 | head -40
fi
exit 0
