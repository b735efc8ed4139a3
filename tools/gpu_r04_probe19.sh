#!/bin/bash
# Round 4: k_extend at 5 waves per SIMD (libigx_E5.so, -DEXTEND_WAVES=5: 96
# VGPRs) against 4 on the global-table fused scenes, interleaved.
set -o pipefail
mkdir -p gpurun_out/r04l
export TMPDIR=/tmp
O=gpurun_out/r04l
for lib in libigx.so libigx_E5.so libigx.so libigx_E5.so; do
  echo "== $lib" >> $O/ab.log
  IGX_LIB_PATH=$PWD/ignis-masterthesis_amd/$lib timeout -k 10 300 python3 tools/sweep_frame.py scenes/s_deep.json '[{}]' 16 >> $O/ab.log 2>&1 || exit 1
  IGX_LIB_PATH=$PWD/ignis-masterthesis_amd/$lib timeout -k 10 300 python3 tools/sweep_frame.py scenes/s_deep.json '[{"concurrent_chunks": 0}]' 8 4096x4096 >> $O/ab.log 2>&1 || exit 1
done
cut -c1-140 $O/ab.log
