#!/bin/bash
# Round-4 start: GPU suite on the inherited tree, then S-deep (config-4/5
# stand-in) diagnosis of k_extend: L2 / L1 hit rates, texture-path busy,
# wave-state counters (one rocprofv3 --pmc pass per block set), and the
# instrumented per-ray / per-class statistics.
set -o pipefail
mkdir -p gpurun_out/r04s
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r04s/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/r04s/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 60 rocprofv3 -L > gpurun_out/r04s/counters.txt 2>&1 || true
timeout -k 10 120 python3 tools/ray_stats.py scenes/s_deep.json > gpurun_out/r04s/ray_stats_s_deep.json 2>&1 || exit 1
i=0
for set in "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE" \
           "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TA_BUSY_avr TD_BUSY_avr" \
           "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_THREAD_CYCLES_VALU"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $set -d gpurun_out/r04s/p$i -o run --output-format csv -- python3 tools/pmc_run.py 8 s_deep.json > gpurun_out/r04s/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/r04s/p$i.log; exit 1; }
done
echo done
