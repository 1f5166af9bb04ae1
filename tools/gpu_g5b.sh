set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python tools/gemm_sp_micro.py > gpurun_out/g5_micro2.json 2>gpurun_out/g5_micro.err || { tail -5 gpurun_out/g5_micro.err; exit 1; }
grep group gpurun_out/g5_micro2.json
