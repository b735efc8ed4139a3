#!/bin/bash
# Round 4: the diamond with LDS-staged vs global traversal tables (option
# lds_scene_max; refill auto / off), then the translation-only instance
# shortcut (libigx_T.so, -DIGX_TRANSLATE_INSTANCES=1) against the default.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python3 tools/sweep_frame.py scenes/diamond_scene.json '[{"lds_scene_max": 49152}, {"lds_scene_max": 0}, {"lds_scene_max": 0, "refill": 0}, {"lds_scene_max": 49152, "refill": -1}, {"lds_scene_max": 0, "refill": -1}]' 32 > gpurun_out/lds_ab.log 2>&1 || { tail -5 gpurun_out/lds_ab.log; exit 1; }
cut -c1-140 gpurun_out/lds_ab.log
bash tools/ab_libs.sh "libigx.so libigx_T.so" scenes/diamond_scene.json > gpurun_out/ab_translate.log 2>&1
