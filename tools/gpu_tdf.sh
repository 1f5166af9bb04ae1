set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_engine_gpu.py tests/test_split_gpu.py tests/test_actor_gpu.py tests/test_native_gpu.py > gpurun_out/tdf_tests.txt 2>&1 || { tail -30 gpurun_out/tdf_tests.txt; exit 1; }
tail -1 gpurun_out/tdf_tests.txt
for r in 1 2; do
for v in 1 0; do
timeout -k 10 200 python bench.py --steps 300 --set learner.td_fuse_head_fwd=$v > gpurun_out/tdf_b$v.log 2>&1 || exit 1
echo "fuse_fwd=$v $(grep -h metric gpurun_out/tdf_b$v.log | cut -c1-60)"
done
done
timeout -k 10 200 python bench.py --steps 200 --dtype bf16 > gpurun_out/tdf_bf16.log 2>&1 || exit 1
echo "bf16 $(grep -h metric gpurun_out/tdf_bf16.log | cut -c1-60)"
