#!/bin/bash
# PMC: VALU busy / utilisation, wave cycles and L2 hit rate of the traversal
# kernels on one scene.  usage: gpu_pmc_valu.sh scene.json '{"split": 1}'
set -o pipefail
mkdir -p gpurun_out/valu
export TMPDIR=/tmp
SC=${1:-s_soup_16m.json}; OPT=${2:-'{}'}
i=0
for set in "SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_THREAD_CYCLES_VALU GRBM_GUI_ACTIVE" \
           "TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr TD_BUSY_avr GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $set -d gpurun_out/valu/p$i -o run --output-format csv -- python3 tools/pmc_run.py 1 $SC "$OPT" > gpurun_out/valu/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/valu/p$i.log; exit 1; }
done
echo done
