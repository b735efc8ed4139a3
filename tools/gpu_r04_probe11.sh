#!/bin/bash
# Round 4: concurrent chunks (libigx_C.so, option concurrent_chunks) against
# the sequential schedule on the same library, interleaved: frames and image
# md5 on the diamond, primitives, S-deep at 1000^2 and 4096^2; then the GPU
# suite on libigx_C.so (concurrent by default).
set -o pipefail
mkdir -p gpurun_out/r04c
export TMPDIR=/tmp
O=gpurun_out/r04c
export IGX_LIB_PATH=$PWD/ignis-masterthesis_amd/libigx_C.so
AB='[{"concurrent_chunks": 0}, {"concurrent_chunks": 1}, {"concurrent_chunks": 0}, {"concurrent_chunks": 1}]'
timeout -k 10 300 python3 tools/sweep_frame.py scenes/diamond_scene.json "$AB" 32 > $O/ab.log 2>&1 || { tail -5 $O/ab.log; exit 1; }
timeout -k 10 300 python3 tools/sweep_frame.py scenes/primitives.json "$AB" 32 >> $O/ab.log 2>&1 || { tail -5 $O/ab.log; exit 1; }
timeout -k 10 300 python3 tools/sweep_frame.py scenes/s_deep.json "$AB" 16 >> $O/ab.log 2>&1 || { tail -5 $O/ab.log; exit 1; }
timeout -k 10 400 python3 tools/sweep_frame.py scenes/s_deep.json "$AB" 8 4096x4096 >> $O/ab.log 2>&1 || { tail -5 $O/ab.log; exit 1; }
cut -c1-190 $O/ab.log
timeout -k 10 700 python3 -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; exit $rc
