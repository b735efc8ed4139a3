#!/bin/bash
# Quick GPU-box session: gpu tests, smoke, one default bench line.  Each GPU step
# has its own time limit; the chain stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && tail -3 gpurun_out/pytest_gpu.log && \
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && tail -2 gpurun_out/smoke.log && \
timeout -k 10 600 python3 bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err && cat gpurun_out/bench.json
rc=$?
echo "rc=$rc"
exit $rc
