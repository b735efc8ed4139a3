#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python3 tools/sweep_frame.py scenes/diamond_scene.json '[{"inline_shadow":1},{"inline_shadow":0},{"inline_shadow":1},{"inline_shadow":0}]' 32 > gpurun_out/exp_i.log 2>&1
rc=$?; cut -c1-250 gpurun_out/exp_i.log; exit $rc
