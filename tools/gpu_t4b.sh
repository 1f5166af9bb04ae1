set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_split_gpu.py tests/test_kernels_gpu.py tests/test_engine_gpu.py > gpurun_out/t4b_tests.txt 2>&1 || { tail -30 gpurun_out/t4b_tests.txt; exit 1; }
tail -1 gpurun_out/t4b_tests.txt
for r in 1 2; do
for v in 1 0; do
timeout -k 10 200 python bench.py --steps 300 --set learner.lstm_tag_words=$v > gpurun_out/t4b_b$v.log 2>&1 || exit 1
echo "words=$v $(grep -h metric gpurun_out/t4b_b$v.log | cut -c1-60)"
done
done
bash tools/prof_bench.sh fp32_t4b || exit 1
