#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
T='[{"bvh_quantize":1},{"bvh_quantize":0},{"bvh_quantize":1},{"bvh_quantize":0}]'
timeout -k 10 200 python3 tools/sweep_frame.py scenes/primitives.json "$T" 8 > gpurun_out/exp_k.log 2>&1 && \
timeout -k 10 300 python3 tools/sweep_frame.py scenes/s_deep.json "$T" 8 >> gpurun_out/exp_k.log 2>&1 && \
timeout -k 10 300 python3 tools/sweep_frame.py scenes/s_soup_1m.json "$T" 2 >> gpurun_out/exp_k.log 2>&1 && \
timeout -k 10 400 python3 tools/sweep_frame.py scenes/s_soup_16m.json "$T" 1 >> gpurun_out/exp_k.log 2>&1
rc=$?; cut -c1-250 gpurun_out/exp_k.log; exit $rc
