#!/bin/bash
# Is the traversal bound by the vector-memory address path (TA/TD)?
set -o pipefail
mkdir -p gpurun_out/ta
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --pmc TA_BUSY_avr TA_BUSY_max GRBM_GUI_ACTIVE -d gpurun_out/ta/p1 -o run --output-format csv -- python3 tools/pmc_run.py 1 > gpurun_out/ta/p1.log 2>&1 && \
timeout -k 10 240 rocprofv3 --pmc TD_TD_BUSY_sum TA_TOTAL_WAVEFRONTS_sum TCP_PENDING_STALL_CYCLES_sum -d gpurun_out/ta/p2 -o run --output-format csv -- python3 tools/pmc_run.py 1 > gpurun_out/ta/p2.log 2>&1 && \
timeout -k 10 240 rocprofv3 --kernel-trace -d gpurun_out/ta/kt -o run --output-format csv -- python3 tools/pmc_run.py 1 > gpurun_out/ta/kt.log 2>&1
echo rc=$?
