#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
T='[{"overlap_shadow":1},{"overlap_shadow":0},{"overlap_shadow":1},{"overlap_shadow":0}]'
timeout -k 10 300 python3 tools/sweep_frame.py scenes/s_soup_16m.json "$T" 1 > gpurun_out/exp_f16.log 2>&1 && \
timeout -k 10 300 python3 tools/sweep_frame.py scenes/s_soup_1m.json "$T" 2 > gpurun_out/exp_f1.log 2>&1 && \
cut -c1-230 gpurun_out/exp_f16.log gpurun_out/exp_f1.log && \
timeout -k 10 900 python3 -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log; exit $rc
