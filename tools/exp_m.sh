#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 tools/sweep_frame.py scenes/s_soup_16m.json '[{},{"bvh_quantize":0}]' 1 > gpurun_out/exp_m.log 2>&1; rc=$?
cut -c1-250 gpurun_out/exp_m.log; exit $rc
