#!/bin/bash
# Round 4: S-soup-16M trace kernel alone (overlap_shadow 0): refill threshold
# (option refill) and BLAS leaf size (bvh_leaf_size, re-upload), and the
# persistent-lane kernels at 7 waves per SIMD (libigx_W7.so) against 6.
set -o pipefail
mkdir -p gpurun_out/r04k
export TMPDIR=/tmp
O=gpurun_out/r04k
timeout -k 10 500 python3 tools/sweep_frame.py scenes/s_soup_16m.json '[{"overlap_shadow": 0}, {"refill": 8}, {"refill": 24}, {"refill": 32}, {"refill": 16}, {"bvh_leaf_size": 2}, {"bvh_leaf_size": 1}, {"bvh_leaf_size": 4}]' 1 > $O/soup16_opts.log 2>&1 || { tail -5 $O/soup16_opts.log; exit 1; }
cut -c1-150 $O/soup16_opts.log
for lib in libigx.so libigx_W7.so libigx.so libigx_W7.so; do
  IGX_LIB_PATH=$PWD/ignis-masterthesis_amd/$lib timeout -k 10 300 python3 tools/sweep_frame.py scenes/s_soup_16m.json '[{"overlap_shadow": 0}]' 1 >> $O/soup16_w7.log 2>&1 || exit 1
  echo "== $lib" >> $O/soup16_w7.log
done
cut -c1-150 $O/soup16_w7.log
