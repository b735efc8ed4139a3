#!/bin/bash
# Round 4: consistency of the instrumented k_extend's per-class node-loop
# iteration counts with the global count: with tail_threshold 0 every
# closest-hit node step runs in k_extend, so the class sums must equal it.
set -o pipefail
mkdir -p gpurun_out/r04n
O=gpurun_out/r04n
timeout -k 10 200 python3 tools/ray_stats.py scenes/s_deep.json '{"tail_threshold": 0}' > $O/sdeep_t0.json 2>&1 || { tail -3 $O/sdeep_t0.json; exit 1; }
timeout -k 10 200 python3 tools/ray_stats.py scenes/diamond_scene.json '{"tail_threshold": 0}' > $O/diamond_t0.json 2>&1 || { tail -3 $O/diamond_t0.json; exit 1; }
timeout -k 10 200 python3 tools/ray_stats.py scenes/diamond_scene.json > $O/diamond.json 2>&1 || { tail -3 $O/diamond.json; exit 1; }
tail -c 1500 $O/sdeep_t0.json
