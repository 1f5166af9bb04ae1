set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_split_gpu.py tests/test_actor_gpu.py -k "fp32 or split or dp or torso" > gpurun_out/split_tests.txt 2>&1 || { tail -30 gpurun_out/split_tests.txt; exit 1; }
tail -2 gpurun_out/split_tests.txt
bash tools/prof_cfg.sh fp4 || exit 1
timeout -k 10 200 python bench.py --steps 100 --warmup 10 > gpurun_out/bench_fp32.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --steps 100 --warmup 10 --set learner.sp_head_grads_in_bptt=false > gpurun_out/bench_fp32_nohg.log 2>&1 || exit 1
grep -h metric gpurun_out/bench_fp32.log gpurun_out/bench_fp32_nohg.log | cut -c1-100
