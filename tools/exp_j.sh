#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python3 tools/sweep_frame.py scenes/diamond_scene.json '[{},{"dynamic":15},{},{"dynamic":15}]' 32 > gpurun_out/exp_j.log 2>&1 && \
timeout -k 10 200 python3 tools/sweep_frame.py scenes/primitives.json '[{},{"dynamic":15},{},{"dynamic":15}]' 8 >> gpurun_out/exp_j.log 2>&1
rc=$?; cut -c1-250 gpurun_out/exp_j.log; exit $rc
