#!/bin/bash
# PMC counters of every kernel of the fp32 learner step (bench.py, graph replay), one counter
# group per rocprofv3 pass (kernel-trace only) -> gpurun_out/pmc_step/summary.txt
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_step
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_ACTIVE_INST_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_VALU_MFMA_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU" \
           "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d gpurun_out/pmc_step/p$i -- python bench.py --steps 3 --warmup 2 > gpurun_out/pmc_step/p$i.log 2>&1 || { echo "pass $i rc=$?"; tail -5 gpurun_out/pmc_step/p$i.log; exit 1; }
done
python tools/pmc_summary.py "gpurun_out/pmc_step/p*/**/*counter_collection.csv" torso lstm gemm td_duel rmsprop > gpurun_out/pmc_step/summary.txt
head -150 gpurun_out/pmc_step/summary.txt
