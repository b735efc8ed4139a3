#!/bin/bash
# Round 4: identity-instance shortcut -- GPU suite on the default build, then
# the A/B against the build without it (libigx_A.so, -DIGX_IDENTITY_INSTANCES=0).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python3 -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/pytest_gpu.log | head -20; exit $rc; }
bash tools/ab_libs.sh "libigx.so libigx_A.so" scenes/diamond_scene.json scenes/primitives.json > gpurun_out/ab_ident2.log 2>&1
