#!/bin/bash
# Measurement of record (round 4), part 1: full GPU test suite, bench
# (headline + suite + CPU baseline + config-5 line), rocprofv3 kernel stats of
# the headline (--isolated 0: the timed frames' dispatches only, as the bench's
# HIP events see them) and PMC FETCH_SIZE / WRITE_SIZE of the headline workload.
# Part 2 (suite profiles): tools/gpu_r04_final2.sh.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/prof gpurun_out/pmc_fetch gpurun_out/pmc_write
timeout -k 10 700 python3 -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 600 python3 bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err && head -c 400 gpurun_out/bench.json && echo && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --suite 0 --config5 0 --isolated 0 > gpurun_out/prof_bench.json 2> gpurun_out/prof.err && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- python3 tools/pmc_run.py 32 > gpurun_out/pmc_fetch.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- python3 tools/pmc_run.py 32 > gpurun_out/pmc_write.log 2>&1
rc=$?; echo "rc=$rc"; exit $rc
