#!/bin/bash
# GPU tests + a diamond frame A/B (shadow classes) on the current tree
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python3 tools/sweep_frame.py scenes/diamond_scene.json '[{"shadow_classes":1},{"shadow_classes":0},{"shadow_classes":1},{"shadow_classes":0}]' 32 > gpurun_out/exp_c_diamond.log 2>&1 && cut -c1-200 gpurun_out/exp_c_diamond.log && \
timeout -k 10 900 python3 -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_gpu.log; grep -E "FAIL|Error" gpurun_out/pytest_gpu.log | head -20; exit $rc
