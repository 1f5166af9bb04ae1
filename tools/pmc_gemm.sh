#!/bin/bash
# PMC counter passes (kernel-trace only, one group per pass) for tools/gemm_pmc.py VERSION SHAPE
export TMPDIR=/tmp
mkdir -p gpurun_out/pmcg
V=${1:-5}; S=${2:-xp2}
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_ACTIVE_INST_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_VALU_MFMA_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU" \
           "SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_WAVES" \
           "TA_BUSY_avr TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d gpurun_out/pmcg/v${V}_${S}_p$i -- python tools/gemm_pmc.py $V 5 $S > gpurun_out/pmcg/v${V}_${S}_p$i.log 2>&1 || { echo "pass $i rc=$?"; tail -5 gpurun_out/pmcg/v${V}_${S}_p$i.log; exit 1; }
done
echo done
