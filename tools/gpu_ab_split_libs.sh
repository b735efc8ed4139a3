#!/bin/bash
# A/B of library builds on the split-schedule soups with overlap_shadow 0
# (trace and shadow kernel times apart), interleaved twice; fb_md5 shows
# whether the images stay identical.  usage: gpu_ab_split_libs.sh lib ...
set -o pipefail
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
O=gpurun_out/ab
for round in 1 2; do for lib in "$@"; do
  for sc in s_soup_1m:2 s_soup_16m:1; do
    echo "== $lib $sc" >> $O/ab.log
    IGX_LIB_PATH=$PWD/ignis-masterthesis_amd/$lib timeout -k 10 300 python3 tools/sweep_frame.py scenes/${sc%%:*}.json '[{"overlap_shadow": 0}]' ${sc##*:} >> $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
  done
done; done
cut -c1-150 $O/ab.log
