#!/bin/bash
# GPU session for the committed profiles: tests, smoke, bench, rocprof kernel
# stats (diamond and S-soup-16M) and the PMC HBM traffic passes.  Every GPU
# step has its own time limit; the chain stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/prof gpurun_out/prof_soup gpurun_out/pmc_* gpurun_out/cal_*
timeout -k 10 900 python3 -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && tail -3 gpurun_out/pytest_gpu.log && \
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && tail -2 gpurun_out/smoke.log && \
timeout -k 10 600 python3 bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err && cat gpurun_out/bench.json && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --suite 0 > gpurun_out/prof_bench.json 2> gpurun_out/prof.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_soup -o run --output-format csv -- python3 tools/pmc_run.py 1 s_soup_16m.json > gpurun_out/prof_soup.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- python3 tools/pmc_run.py 32 > gpurun_out/pmc_fetch.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- python3 tools/pmc_run.py 32 > gpurun_out/pmc_write.log 2>&1 && \
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch_soup -o run --output-format csv -- python3 tools/pmc_run.py 1 s_soup_16m.json > gpurun_out/pmc_fetch_soup.log 2>&1 && \
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write_soup -o run --output-format csv -- python3 tools/pmc_run.py 1 s_soup_16m.json > gpurun_out/pmc_write_soup.log 2>&1
rc=$?
echo "rc=$rc"
exit $rc
