#!/bin/bash
# Round 4: the new GPU tests alone (cycles-box, igcli camera options, imported
# one-leaf BLAS with infinite tmax)
set -o pipefail
mkdir -p gpurun_out/r04t
timeout -k 10 300 python3 -u -m pytest tests/test_eval.py tests/test_gpu.py -x -v -m gpu --timeout 120 --timeout-method thread \
  -k "cycles_box or igcli or one_leaf" > gpurun_out/r04t/pytest_new.log 2>&1
rc=$?; tail -8 gpurun_out/r04t/pytest_new.log; exit $rc
