#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python3 tools/sweep_frame.py scenes/diamond_scene.json '[{"enclosing":1},{"enclosing":0},{"enclosing":1},{"enclosing":0}]' 32 > gpurun_out/exp_e.log 2>&1 && cut -c1-200 gpurun_out/exp_e.log && \
timeout -k 10 900 python3 -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log; exit $rc
