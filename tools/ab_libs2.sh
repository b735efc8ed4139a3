#!/bin/bash
# A/B of library builds under option sets: one bench frame per scene, library
# and option set (tools/sweep_frame.py, best of 2 reps), libraries interleaved
# twice; fb_md5 shows whether the images are identical.
# usage: ab_libs2.sh "libigx.so libigx_B.so" 'OPTIONS_JSON_LIST' ITERATIONS scenes/a.json [...]
set -o pipefail
mkdir -p gpurun_out
LIBS="$1"; OPTS="$2"; IT="$3"; shift 3
for sc in "$@"; do
  for round in 1 2; do
    for lib in $LIBS; do
      echo "== $lib $sc"
      IGX_LIB_PATH=$PWD/ignis-masterthesis_amd/$lib timeout -k 10 300 python3 tools/sweep_frame.py $sc "$OPTS" $IT || exit 1
    done
  done
done
