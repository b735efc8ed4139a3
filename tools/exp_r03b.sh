#!/bin/bash
# A/B: LDS treelet (global-table scenes) and shadow-ray classes (diamond)
set -o pipefail
mkdir -p gpurun_out
T='[{"treelet":-1,"treelet_kernels":7},{"treelet":0},{"treelet":-1,"treelet_kernels":5},{"treelet":-1,"treelet_kernels":7},{"treelet":0},{"treelet":-1,"treelet_kernels":5}]'
timeout -k 10 200 python3 tools/sweep_frame.py scenes/diamond_scene.json '[{"shadow_classes":1},{"shadow_classes":0},{"shadow_classes":1},{"shadow_classes":0},{"bvh_width":4},{"bvh_width":2}]' 32 > gpurun_out/exp_b_diamond.log 2>&1 && \
timeout -k 10 200 python3 tools/sweep_frame.py scenes/primitives.json "$T" 8 > gpurun_out/exp_b_prim.log 2>&1 && \
timeout -k 10 300 python3 tools/sweep_frame.py scenes/s_deep.json "$T" 8 > gpurun_out/exp_b_sdeep.log 2>&1 && \
timeout -k 10 300 python3 tools/sweep_frame.py scenes/s_soup_1m.json "$T" 4 > gpurun_out/exp_b_soup1m.log 2>&1 && \
timeout -k 10 300 python3 tools/sweep_frame.py scenes/s_soup_16m.json "$T" 2 > gpurun_out/exp_b_soup16m.log 2>&1
rc=$?; for f in diamond prim sdeep soup1m soup16m; do echo "== $f"; cut -c1-220 gpurun_out/exp_b_$f.log; done; exit $rc
