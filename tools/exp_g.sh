#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
T='[{"speculative":1},{"speculative":0},{"speculative":1},{"speculative":0}]'
timeout -k 10 300 python3 tools/sweep_frame.py scenes/s_soup_16m.json "$T" 1 > gpurun_out/exp_g16.log 2>&1 && \
timeout -k 10 300 python3 tools/sweep_frame.py scenes/s_soup_1m.json "$T" 2 > gpurun_out/exp_g1.log 2>&1
rc=$?; cut -c1-230 gpurun_out/exp_g16.log gpurun_out/exp_g1.log; exit $rc
