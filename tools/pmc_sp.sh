#!/bin/bash
# PMC counters of the split-precision torso forward + fused x-projection GEMM (tools/sp_micro.py),
# one counter group per rocprofv3 pass (kernel-trace only) -> gpurun_out/pmc_sp/
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_sp
timeout -k 10 120 python tools/sp_micro.py both 20 > gpurun_out/pmc_sp/micro.json 2>&1 || exit $?
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_ACTIVE_INST_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_VALU_MFMA_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_LDS_STORE SQ_INSTS_LDS_LOAD SQ_WAIT_INST_ANY" \
           "SQ_INST_CYCLES_VMEM SQ_INSTS_SALU SQ_ACTIVE_INST_ANY SQ_WAVES" \
           "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d gpurun_out/pmc_sp/p$i -- python tools/sp_micro.py both 3 > gpurun_out/pmc_sp/p$i.log 2>&1 || { echo "pass $i rc=$?"; tail -5 gpurun_out/pmc_sp/p$i.log; exit 1; }
done
python tools/pmc_summary.py "gpurun_out/pmc_sp/p*/**/*counter_collection.csv" torso_fwd_sp gemm5 > gpurun_out/pmc_sp/summary.txt
cat gpurun_out/pmc_sp/micro.json
cat gpurun_out/pmc_sp/summary.txt
