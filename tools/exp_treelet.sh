#!/bin/bash
# A/B of the LDS treelet (option "treelet": -1 auto, 0 off; "treelet_kernels" bits) on the global-table scenes
set -o pipefail
mkdir -p gpurun_out
T='[{"treelet":-1,"treelet_kernels":7},{"treelet":0},{"treelet":-1,"treelet_kernels":5},{"treelet":-1,"treelet_kernels":7},{"treelet":0},{"treelet":-1,"treelet_kernels":5}]'
timeout -k 10 200 python3 tools/sweep_frame.py scenes/primitives.json "$T" 8 > gpurun_out/exp_tree_prim.log 2>&1 && \
timeout -k 10 300 python3 tools/sweep_frame.py scenes/s_deep.json "$T" 8 > gpurun_out/exp_tree_sdeep.log 2>&1 && \
timeout -k 10 300 python3 tools/sweep_frame.py scenes/s_soup_1m.json "$T" 4 > gpurun_out/exp_tree_soup1m.log 2>&1 && \
timeout -k 10 300 python3 tools/sweep_frame.py scenes/s_soup_16m.json "$T" 2 > gpurun_out/exp_tree_soup16m.log 2>&1
rc=$?; for f in prim sdeep soup1m soup16m; do echo "== $f"; cut -c1-200 gpurun_out/exp_tree_$f.log; done; exit $rc
