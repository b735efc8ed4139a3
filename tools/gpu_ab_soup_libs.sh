#!/bin/bash
# A/B of library builds on the two soups (split schedule), interleaved twice.
# usage: gpu_ab_soup_libs.sh "libigx.so libigx_B.so ..."
set -o pipefail
mkdir -p gpurun_out
for round in 1 2; do for lib in $1; do
  export IGX_LIB_PATH=$PWD/ignis-masterthesis_amd/$lib; echo "== $lib"
  timeout -k 10 200 python3 tools/sweep_frame.py scenes/s_soup_1m.json '[{}]' 8 || exit 1
  if [ $round = 1 ]; then timeout -k 10 300 python3 tools/sweep_frame.py scenes/s_soup_16m.json '[{}]' 2 || exit 1; fi
done; done
