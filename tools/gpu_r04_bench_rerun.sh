#!/bin/bash
# Round 4: bench.py once more with the round-4 profiles committed (its suite
# lines cite them), then the chunk-size experiment under concurrent chunks.
set -o pipefail
mkdir -p gpurun_out/r04j
export TMPDIR=/tmp
timeout -k 10 600 python3 bench.py > gpurun_out/r04j/bench.json 2> gpurun_out/r04j/bench.err || { tail -5 gpurun_out/r04j/bench.err; exit 1; }
head -c 300 gpurun_out/r04j/bench.json; echo
bash tools/gpu_r04_probe14.sh
