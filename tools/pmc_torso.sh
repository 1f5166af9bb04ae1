#!/bin/bash
# PMC counters for the torso kernels, one counter group per rocprofv3 pass (kernel-trace only).
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
python -c "import __graft_entry__ as g; g.build()" > /dev/null || exit 1
timeout -k 10 120 python tools/torso_micro.py both 20 > gpurun_out/pmc/micro.json 2>&1 || exit $?
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_ACTIVE_INST_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_VALU_MFMA_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_LDS_STORE SQ_INSTS_LDS_LOAD SQ_WAIT_INST_ANY" \
           "SQ_LDS_UNALIGNED_STALL SQ_INSTS_SALU SQ_INST_CYCLES_VMEM SQ_WAVES"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d gpurun_out/pmc/p$i -- python tools/torso_micro.py both 3 > gpurun_out/pmc/p$i.log 2>&1 || { echo "pass $i rc=$?"; exit 1; }
done
echo done
