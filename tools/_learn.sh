# memory-task stored-state protocol: 2 seeds x {full, zero_state, memoryless}, switch 64
set -o pipefail
mkdir -p gpurun_out/learn
for seed in 0 1; do
  for arm in none zero_state memoryless; do
    timeout -k 10 400 python -u tools/learn_check.py --memory --switch 64 --episode-len 128 \
      --burn-in 4 --learn 8 --steps 8000 --ablation $arm --seed $seed \
      > gpurun_out/learn/${arm}_${seed}.log 2>&1 || { tail -20 gpurun_out/learn/${arm}_${seed}.log; exit 1; }
    echo "$arm seed $seed: $(grep -h '^{' gpurun_out/learn/${arm}_${seed}.log | tail -1 | cut -c1-400)"
  done
done
