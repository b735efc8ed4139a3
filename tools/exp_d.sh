#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python3 tools/sweep_frame.py scenes/diamond_scene.json '[{"path_classes":3},{"path_classes":1,"shadow_classes":0},{"path_classes":3,"shadow_classes":1},{"path_classes":1,"shadow_classes":0}]' 32 > gpurun_out/exp_d.log 2>&1 && \
timeout -k 10 200 python3 tools/ray_stats.py scenes/diamond_scene.json '{"path_classes":3}' > gpurun_out/rs3b.json 2>&1
rc=$?; cut -c1-200 gpurun_out/exp_d.log; cat gpurun_out/rs3b.json; exit $rc
