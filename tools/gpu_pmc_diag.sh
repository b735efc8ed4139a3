#!/bin/bash
# PMC diagnosis of k_extend: wave-state and cache counters in separate passes.
set -o pipefail
mkdir -p gpurun_out/diag
export TMPDIR=/tmp
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS" \
           "SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM" \
           "TCC_HIT_sum TCC_MISS_sum" "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $set -d gpurun_out/diag/p$i -o run --output-format csv -- python3 tools/pmc_run.py 1 > gpurun_out/diag/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/diag/p$i.log; exit 1; }
done
echo done
