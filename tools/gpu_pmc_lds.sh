#!/bin/bash
# PMC: LDS instruction mix, bank conflicts and LDS waits of the kernels of one scene.
# usage: gpu_pmc_lds.sh scene.json '{options}'
set -o pipefail
mkdir -p gpurun_out/lds
export TMPDIR=/tmp
SC=${1:-diamond_scene.json}; OPT=${2:-'{}'}
timeout -k 10 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE \
  -d gpurun_out/lds/p1 -o run --output-format csv -- python3 tools/pmc_run.py 4 $SC "$OPT" > gpurun_out/lds/p1.log 2>&1 || { tail -5 gpurun_out/lds/p1.log; exit 1; }
echo done
