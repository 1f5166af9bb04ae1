#!/bin/bash
# Instruction budget of the fp32 torso forward (torso_fwd_sp2_kernel) by phase (round-6 verdict
# item 2): tools/torso_lds_variants.py's dbg-bit variants under two PMC passes (8 SQ counters
# each), summarized per variant.  Run through gpurun from the repo root.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/tbud
i=0
for grp in "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT"; do
  i=$((i+1))
  rm -rf gpurun_out/tbud/p$i
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d gpurun_out/tbud/p$i -- \
    python tools/torso_lds_variants.py > gpurun_out/tbud/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/tbud/p$i.log; exit 1; }
  python tools/torso_lds_variants.py --summarize "gpurun_out/tbud/p$i/*/*counter_collection.csv" > gpurun_out/tbud/s$i.txt
done
cat gpurun_out/tbud/s1.txt gpurun_out/tbud/s2.txt
