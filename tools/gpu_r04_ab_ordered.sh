#!/bin/bash
# Round 4: octant-ordered slab tests (libigx_O.so, -DIGX_ORDERED_SLAB=1)
# against the default build: frames of the 4-wide and quantised scenes
# (fb_md5 equal = same image), then the ordered build's GPU parity tests.
set -o pipefail
mkdir -p gpurun_out/r04o
export TMPDIR=/tmp
O=gpurun_out/r04o
for round in 1 2; do for lib in libigx.so libigx_O.so; do
  export IGX_LIB_PATH=$PWD/ignis-masterthesis_amd/$lib; echo "== $lib" | tee -a $O/ab.log
  timeout -k 10 200 python3 tools/sweep_frame.py scenes/s_deep.json '[{}]' 16 >> $O/ab.log 2>&1 || exit 1
  timeout -k 10 200 python3 tools/sweep_frame.py scenes/primitives.json '[{}]' 32 >> $O/ab.log 2>&1 || exit 1
  timeout -k 10 200 python3 tools/sweep_frame.py scenes/s_soup_1m.json '[{}]' 8 >> $O/ab.log 2>&1 || exit 1
  timeout -k 10 300 python3 tools/sweep_frame.py scenes/s_soup_16m.json '[{}]' 1 >> $O/ab.log 2>&1 || exit 1
done; done
cut -c1-200 $O/ab.log
[ "$1" = tests ] || exit 0
export IGX_LIB_PATH=$PWD/ignis-masterthesis_amd/libigx_O.so
timeout -k 10 900 python3 -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -rA > $O/pytest_gpu_O.log 2>&1
rc=$?; tail -3 $O/pytest_gpu_O.log; exit $rc
