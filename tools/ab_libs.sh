#!/bin/bash
# A/B of library builds (make BUILD=build_X LIB=libigx_X.so EXTRA=...): one
# bench frame per scene and library (tools/sweep_frame.py, best of 2 reps),
# libraries interleaved twice; fb_md5 shows whether the images are identical.
# usage: ab_libs.sh "libigx.so libigx_B.so" [scene.json ...]
set -o pipefail
mkdir -p gpurun_out
LIBS="$1"; shift
SCENES=${@:-scenes/diamond_scene.json}
for sc in $SCENES; do
  for round in 1 2; do
    for lib in $LIBS; do
      echo "== $lib $sc"
      IGX_LIB_PATH=$PWD/ignis-masterthesis_amd/$lib timeout -k 10 300 python3 tools/sweep_frame.py $sc '[{}]' 32 || exit 1
    done
  done
done
