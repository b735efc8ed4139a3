#!/bin/bash
# Measurement of record (round 4), part 2: rocprof + PMC profiles of every
# suite line (tools/gpu_profile_suite.sh) and the 2-rank rehearsal through the
# launcher (both lines, frame check).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_profile_suite.sh && \
IGX_BENCH_REHEARSAL=1 timeout -k 10 600 python3 bench.py --gpus 2 --steps 2 --warmup 1 --config5-steps 1 > gpurun_out/rehearse2.json 2> gpurun_out/rehearse2.err
rc=$?; echo "rc=$rc"; exit $rc
