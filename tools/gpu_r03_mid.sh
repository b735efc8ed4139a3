#!/bin/bash
# Mid-round measurement: bench (headline + suite), instrumented ray statistics
# of the diamond under the path-class options, rocprof kernel stats and PMC
# traffic of the headline workload.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/prof gpurun_out/pmc_fetch gpurun_out/pmc_write
timeout -k 10 600 python3 bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err && head -c 600 gpurun_out/bench.json && echo && \
timeout -k 10 200 python3 tools/ray_stats.py scenes/diamond_scene.json '{"path_classes":3}' > gpurun_out/rs3.json 2>&1 && \
timeout -k 10 200 python3 tools/ray_stats.py scenes/diamond_scene.json '{"path_classes":1,"shadow_classes":0}' > gpurun_out/rs1.json 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --suite 0 > gpurun_out/prof_bench.json 2> gpurun_out/prof.err && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- python3 tools/pmc_run.py 32 > gpurun_out/pmc_fetch.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- python3 tools/pmc_run.py 32 > gpurun_out/pmc_write.log 2>&1
rc=$?; cat gpurun_out/rs3.json gpurun_out/rs1.json; echo "rc=$rc"; exit $rc
