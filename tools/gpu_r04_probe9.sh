#!/bin/bash
# Round 4: kernel timeline of the diamond's N = 8 rank frame (two handles
# alternating, tools/rank_pipeline.py) and of the N = 1 frame, to see where the
# 8-rank frame's 3 ms over 1/8 of the single-GPU frame go.
set -o pipefail
mkdir -p gpurun_out/r04y
export TMPDIR=/tmp
O=gpurun_out/r04y
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/n8 -o run --output-format csv -- python3 tools/rank_pipeline.py scenes/diamond_scene.json 8 6 1 > $O/n8.log 2>&1 || { tail -5 $O/n8.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/n1 -o run --output-format csv -- python3 tools/rank_pipeline.py scenes/diamond_scene.json 1 3 2 > $O/n1.log 2>&1 || { tail -5 $O/n1.log; exit 1; }
grep '^{' $O/n8.log $O/n1.log | cut -c1-300
