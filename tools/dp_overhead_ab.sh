set -o pipefail
run() { timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 2954$1 bench.py --steps 300 --warmup 30 --force-dp "${@:2}" > gpurun_out/dpab_$1.log 2>&1 || { tail -5 gpurun_out/dpab_$1.log; exit 1; }; echo "[$*] $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/dpab_$1.log)"; }
run 1
run 2 --set dist.comm_reserve_cus=0
run 3 --set dist.global_sampling=0
run 4 --set dist.global_sampling=0 --set dist.comm_reserve_cus=0
run 5 --set dist.graph_collectives=1
run 6
timeout -k 10 200 python bench.py --steps 300 --warmup 30 > gpurun_out/dpab_plain.log 2>&1 && echo "[plain] $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/dpab_plain.log)"
