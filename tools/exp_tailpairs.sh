#!/bin/bash
# A/B of the lane-pair tail kernel (option "tail_pairs") on global-table scenes
set -o pipefail
mkdir -p gpurun_out
T='[{"tail_pairs":1},{"tail_pairs":0},{"tail_pairs":1},{"tail_pairs":0}]'
timeout -k 10 300 python3 tools/sweep_frame.py scenes/s_soup_16m.json "$T" 1 > gpurun_out/exp_tp_soup16m.log 2>&1 && \
timeout -k 10 300 python3 tools/sweep_frame.py scenes/s_soup_1m.json "$T" 2 > gpurun_out/exp_tp_soup1m.log 2>&1 && \
timeout -k 10 300 python3 tools/sweep_frame.py scenes/s_deep.json "$T" 8 > gpurun_out/exp_tp_sdeep.log 2>&1 && \
timeout -k 10 300 python3 tools/sweep_frame.py scenes/materials.json "$T" 8 > gpurun_out/exp_tp_materials.log 2>&1
rc=$?; for f in soup16m soup1m sdeep materials; do echo "== $f"; cut -c1-250 gpurun_out/exp_tp_$f.log; done; exit $rc
