#!/bin/bash
# Round 4 end check of the committed tree as built in-tree: the GPU suite and
# one default bench run (headline, suite lines, CPU baseline).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python3 -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 600 python3 bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err && head -c 600 gpurun_out/bench.json && echo
rc=$?; echo "rc=$rc"; exit $rc
