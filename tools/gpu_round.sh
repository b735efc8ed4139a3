#!/bin/bash
# GPU-box session: tests, smoke, bench, rocprof kernel trace. Each GPU step has its own limit.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python3 -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?" >> gpurun_out/status.txt
tail -5 gpurun_out/pytest_gpu.log
grep -q "passed" gpurun_out/pytest_gpu.log || exit 1
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && tail -2 gpurun_out/smoke.log && \
timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 > gpurun_out/bench.json 2> gpurun_out/bench.err && cat gpurun_out/bench.json && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/prof_bench.json 2> gpurun_out/prof.err; echo "prof rc=$?"
