#!/bin/bash
# Round 4: face records with the vertex normals (libigx_R.so: one dependent
# load fewer in surface_element) against the current library, interleaved;
# fb_md5 must match (same normals, same arithmetic); then the R library's GPU
# suite.
set -o pipefail
mkdir -p gpurun_out/r04o2
export TMPDIR=/tmp
O=gpurun_out/r04o2
for lib in libigx.so libigx_R.so libigx.so libigx_R.so; do
  echo "== $lib" >> $O/ab.log
  IGX_LIB_PATH=$PWD/ignis-masterthesis_amd/$lib timeout -k 10 300 python3 tools/sweep_frame.py scenes/diamond_scene.json '[{}]' 32 >> $O/ab.log 2>&1 || exit 1
  IGX_LIB_PATH=$PWD/ignis-masterthesis_amd/$lib timeout -k 10 300 python3 tools/sweep_frame.py scenes/primitives.json '[{}]' 32 >> $O/ab.log 2>&1 || exit 1
  IGX_LIB_PATH=$PWD/ignis-masterthesis_amd/$lib timeout -k 10 300 python3 tools/sweep_frame.py scenes/materials.json '[{}]' 32 >> $O/ab.log 2>&1 || exit 1
done
cut -c1-140 $O/ab.log
export IGX_LIB_PATH=$PWD/ignis-masterthesis_amd/libigx_R.so
timeout -k 10 700 python3 -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_R.log 2>&1
rc=$?; tail -2 $O/pytest_R.log; exit $rc
