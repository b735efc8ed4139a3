#!/bin/bash
# Full GPU test suite, then the measurement of record (tools/gpu_r03_profile.sh)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/pytest_gpu.log | head -20; exit $rc; }
bash tools/gpu_r03_profile.sh
rc=$?; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 tools/sweep_frame.py scenes/diamond_scene.json '[{"path_classes":4},{"path_classes":5},{"path_classes":4},{"path_classes":5}]' 32 > gpurun_out/exp_q.log 2>&1; cut -c1-200 gpurun_out/exp_q.log
