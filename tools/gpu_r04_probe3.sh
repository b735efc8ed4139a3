#!/bin/bash
# Round 4: GPU suite with the octant-ordered quantised slab test and exit
# widening (libigx.so), then the soups against libigx_O.so (ordered, no
# widening) for the widening's cost.
set -o pipefail
mkdir -p gpurun_out/r04r
export TMPDIR=/tmp
O=gpurun_out/r04r
timeout -k 10 700 python3 -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -rA --durations=15 > $O/pytest_gpu.log 2>&1
rc=$?; tail -22 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for round in 1 2; do for lib in libigx.so libigx_O.so; do
  export IGX_LIB_PATH=$PWD/ignis-masterthesis_amd/$lib; echo "== $lib" >> $O/ab.log
  timeout -k 10 200 python3 tools/sweep_frame.py scenes/s_soup_1m.json '[{}]' 8 >> $O/ab.log 2>&1 || exit 1
  timeout -k 10 300 python3 tools/sweep_frame.py scenes/s_soup_16m.json '[{}]' 1 >> $O/ab.log 2>&1 || exit 1
done; done
cut -c1-150 $O/ab.log
