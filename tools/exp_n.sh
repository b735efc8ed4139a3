#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/exp_n.log
for sc in s_soup_16m s_soup_1m; do
  for lib in libigx.so libigx_B.so libigx.so libigx_B.so; do
    echo "== $lib $sc" >> gpurun_out/exp_n.log
    IGX_LIB_PATH=$PWD/ignis-masterthesis_amd/$lib timeout -k 10 300 python3 tools/sweep_frame.py scenes/$sc.json '[{}]' 1 >> gpurun_out/exp_n.log 2>&1 || exit 1
  done
done
cut -c1-200 gpurun_out/exp_n.log
