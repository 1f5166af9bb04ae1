set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
echo SMOKE ok
timeout -k 10 700 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/pytest_gpu.txt 2>&1 || { tail -30 gpurun_out/pytest_gpu.txt; exit 1; }
tail -1 gpurun_out/pytest_gpu.txt
for c in "atari57" "atari57 --dtype bf16" "atari57 --target-mode shifted" "dmlab30" "seaquest8" "reference"; do
  tag=$(echo $c | tr ' ' '_' | tr -d '-')
  timeout -k 10 200 python bench.py --steps 200 --config $c > gpurun_out/b4_$tag.log 2>&1 || exit 1
  echo "$tag $(grep -h metric gpurun_out/b4_$tag.log | cut -c1-75)"
done
bash tools/prof_bench.sh fp32_r4 || exit 1
