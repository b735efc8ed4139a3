#!/bin/bash
# Measurement of record, part 2: rocprof + PMC profiles of every suite line
# (tools/gpu_profile_suite.sh) and the multi-rank rehearsal through the launcher.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_profile_suite.sh && \
IGX_BENCH_REHEARSAL=1 timeout -k 10 400 python3 bench.py --gpus 4 --steps 2 --warmup 1 --check-frame > gpurun_out/rehearse4.json 2> gpurun_out/rehearse4.err
rc=$?; echo "rc=$rc"; exit $rc
