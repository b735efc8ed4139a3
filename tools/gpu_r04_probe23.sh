#!/bin/bash
# Round 4: kernels built without IEEE-mode min / max (libigx_I.so:
# -mno-amdgpu-ieee -fno-honor-nans, no canonicalising v_max x, x before the
# slab-test min / max) against the default, interleaved; fb_md5 shows whether
# the images stay identical.
set -o pipefail
mkdir -p gpurun_out/r04p2
export TMPDIR=/tmp
O=gpurun_out/r04p2
for lib in libigx.so libigx_I.so libigx.so libigx_I.so; do
  echo "== $lib" >> $O/ab.log
  IGX_LIB_PATH=$PWD/ignis-masterthesis_amd/$lib timeout -k 10 300 python3 tools/sweep_frame.py scenes/s_soup_16m.json '[{"overlap_shadow": 0}]' 1 >> $O/ab.log 2>&1 || exit 1
  IGX_LIB_PATH=$PWD/ignis-masterthesis_amd/$lib timeout -k 10 300 python3 tools/sweep_frame.py scenes/diamond_scene.json '[{}]' 32 >> $O/ab.log 2>&1 || exit 1
  IGX_LIB_PATH=$PWD/ignis-masterthesis_amd/$lib timeout -k 10 300 python3 tools/sweep_frame.py scenes/s_deep.json '[{}]' 16 >> $O/ab.log 2>&1 || exit 1
done
cut -c1-140 $O/ab.log
