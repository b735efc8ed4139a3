#!/bin/bash
# Round 4: fast spherical-rectangle sampler (libigx_F.so, -DIGX_FAST_QUAD=1)
# against the default, interleaved (diamond, S-deep, primitives); then the F
# library's image-parity tests against the oracle and the reference images.
set -o pipefail
mkdir -p gpurun_out/r04m
export TMPDIR=/tmp
O=gpurun_out/r04m
for lib in libigx.so libigx_F.so libigx.so libigx_F.so; do
  echo "== $lib" >> $O/ab.log
  IGX_LIB_PATH=$PWD/ignis-masterthesis_amd/$lib timeout -k 10 300 python3 tools/sweep_frame.py scenes/diamond_scene.json '[{}]' 32 >> $O/ab.log 2>&1 || exit 1
  IGX_LIB_PATH=$PWD/ignis-masterthesis_amd/$lib timeout -k 10 300 python3 tools/sweep_frame.py scenes/s_deep.json '[{}]' 16 >> $O/ab.log 2>&1 || exit 1
  IGX_LIB_PATH=$PWD/ignis-masterthesis_amd/$lib timeout -k 10 300 python3 tools/sweep_frame.py scenes/primitives.json '[{}]' 32 >> $O/ab.log 2>&1 || exit 1
done
cut -c1-140 $O/ab.log
export IGX_LIB_PATH=$PWD/ignis-masterthesis_amd/libigx_F.so
timeout -k 10 700 python3 -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -k "config2 or config3 or config4 or image_parity or eval or area" > $O/pytest_F.log 2>&1
rc=$?; tail -3 $O/pytest_F.log; exit $rc
