#!/bin/bash
# Round-3 measurement of record: bench (headline + suite), rocprof kernel
# stats and PMC traffic of the headline workload, suite profiles (configs 3-5
# and the soups), multi-GPU rehearsal through the launcher.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/prof gpurun_out/pmc_fetch gpurun_out/pmc_write
timeout -k 10 600 python3 bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err && head -c 400 gpurun_out/bench.json && echo && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --suite 0 > gpurun_out/prof_bench.json 2> gpurun_out/prof.err && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- python3 tools/pmc_run.py 32 > gpurun_out/pmc_fetch.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- python3 tools/pmc_run.py 32 > gpurun_out/pmc_write.log 2>&1 && \
bash tools/gpu_profile_suite.sh && \
IGX_BENCH_REHEARSAL=1 timeout -k 10 400 python3 bench.py --gpus 4 --steps 2 --warmup 1 --check-frame > gpurun_out/rehearse4.json 2> gpurun_out/rehearse4.err
rc=$?; echo "rc=$rc"; exit $rc
