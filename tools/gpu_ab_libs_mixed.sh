#!/bin/bash
# A/B of two library builds on the global-table scenes (tools/sweep_frame.py,
# best of 2 reps), libraries interleaved twice; fb_md5 shows whether the
# images are identical.  usage: gpu_ab_libs_mixed.sh "libA.so libB.so"
set -o pipefail
mkdir -p gpurun_out
LIBS=${1:-"libigx.so libigx_B.so"}
for round in 1 2; do
  for lib in $LIBS; do
    export IGX_LIB_PATH=$PWD/ignis-masterthesis_amd/$lib
    echo "== $lib soup-1M / S-deep / primitives / soup-16M"
    timeout -k 10 200 python3 tools/sweep_frame.py scenes/s_soup_1m.json '[{}]' 8 || exit 1
    timeout -k 10 200 python3 tools/sweep_frame.py scenes/s_deep.json '[{}]' 8 || exit 1
    timeout -k 10 200 python3 tools/sweep_frame.py scenes/primitives.json '[{}]' 32 || exit 1
    if [ $round = 1 ]; then timeout -k 10 300 python3 tools/sweep_frame.py scenes/s_soup_16m.json '[{}]' 2 || exit 1; fi
  done
done
