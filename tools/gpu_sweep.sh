#!/bin/bash
# GPU tests, then a tail/capacity sweep of one diamond iteration
mkdir -p gpurun_out
timeout -k 10 400 python3 -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -4 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
OPTS='[{}]'
[ -n "$1" ] && OPTS="$1"
timeout -k 10 300 python3 tools/sweep.py scenes/diamond_scene.json "$OPTS" > gpurun_out/sweep.log 2>&1; rc=$?
cat gpurun_out/sweep.log
exit $rc
