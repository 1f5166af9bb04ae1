#!/bin/bash
# bf16 torso forward: timing + LDS bank-conflict / MFMA PMC passes (kernel-trace only)
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_tb
timeout -k 10 120 python tools/torso_micro.py fwd 20 > gpurun_out/pmc_tb/micro.json 2>&1 || exit $?
i=0
for grp in "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVES" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_VALU_MFMA_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d gpurun_out/pmc_tb/p$i -- python tools/torso_micro.py fwd 3 > gpurun_out/pmc_tb/p$i.log 2>&1 || { echo "pass $i rc=$?"; tail -5 gpurun_out/pmc_tb/p$i.log; exit 1; }
done
python tools/pmc_summary.py "gpurun_out/pmc_tb/p*/**/*counter_collection.csv" torso_fwd > gpurun_out/pmc_tb/summary.txt
cat gpurun_out/pmc_tb/micro.json
cat gpurun_out/pmc_tb/summary.txt
