set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 180 --timeout-method thread tests/test_actor_gpu.py -k "dp_engine" > gpurun_out/dp_tests.txt 2>&1 || { tail -30 gpurun_out/dp_tests.txt; exit 1; }
grep -c PASSED gpurun_out/dp_tests.txt
tail -1 gpurun_out/dp_tests.txt
