#!/bin/bash
# Round-6 limiter evidence: SQ wave-state counters, L2 hit rate and LDS
# counters of one workload (tools/pmc_run.py), one rocprofv3 --pmc pass per
# counter set (each set within gfx950's per-pass slots: <= 8 SQ, <= 4 TCC,
# <= 2 TA / TD / GRBM).  Summarised by tools/pmc_sq_summary.py.
# usage: gpu_pmc_sq.sh TAG ITERATIONS SCENE [OPTIONS_JSON] [SIZE]
set -o pipefail
export TMPDIR=/tmp
TAG=$1; IT=$2; SC=$3; OPT=${4:-'{}'}; SZ=${5:-0}
OUT=gpurun_out/sq_$TAG
rm -rf $OUT; mkdir -p $OUT
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE" \
           "TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr TD_BUSY_avr GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $set -d $OUT/p$i -o run --output-format csv -- \
    python3 tools/pmc_run.py $IT $SC "$OPT" $SZ > $OUT/p$i.log 2>&1 || { echo "sq pass $i of $TAG failed"; tail -5 $OUT/p$i.log; exit 1; }
done
echo "sq $TAG done"
