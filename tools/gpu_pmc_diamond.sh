#!/bin/bash
# PMC passes (one counter set per run) on the headline workload: VALU busy /
# utilisation, wait cycles, LDS bank conflicts, L2 hit rate per kernel
set -o pipefail
mkdir -p gpurun_out/valu
export TMPDIR=/tmp
i=0
for set in "SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_THREAD_CYCLES_VALU GRBM_GUI_ACTIVE" \
           "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
           "TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr TD_BUSY_avr GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set -d gpurun_out/valu/p$i -o run --output-format csv -- python3 tools/pmc_run.py 16 > gpurun_out/valu/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/valu/p$i.log; exit 1; }
done
for i in 1 2 3; do python3 tools/pmc_table.py gpurun_out/valu/p$i/run_counter_collection.csv; done > gpurun_out/valu/table.txt
cat gpurun_out/valu/table.txt
