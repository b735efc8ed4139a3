#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
T='[{"bvh_leaf_size":4},{"bvh_leaf_size":2},{"bvh_leaf_size":1},{"bvh_leaf_size":3},{"bvh_leaf_size":4}]'
timeout -k 10 400 python3 tools/sweep_frame.py scenes/s_soup_1m.json "$T" 2 > gpurun_out/exp_h1.log 2>&1
rc=$?; cut -c1-230 gpurun_out/exp_h1.log; exit $rc
