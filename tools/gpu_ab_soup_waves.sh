#!/bin/bash
# A/B of two library builds on the soups with the trace and shadow kernels
# timed apart (overlap_shadow 0).  usage: gpu_ab_soup_waves.sh "libA.so libB.so"
set -o pipefail
mkdir -p gpurun_out
for round in 1 2; do for lib in $1; do
  export IGX_LIB_PATH=$PWD/ignis-masterthesis_amd/$lib; echo "== $lib"
  timeout -k 10 200 python3 tools/sweep_frame.py scenes/s_soup_1m.json '[{"overlap_shadow":0}]' 8 || exit 1
  if [ $round = 1 ]; then timeout -k 10 300 python3 tools/sweep_frame.py scenes/s_soup_16m.json '[{"overlap_shadow":0}]' 2 || exit 1; fi
done; done
