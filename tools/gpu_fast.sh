#!/bin/bash
# quick GPU iteration: gpu tests + bench (no cpu baseline)
mkdir -p gpurun_out
timeout -k 10 400 python3 -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -4 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err; rc=$?
cat gpurun_out/bench.json; tail -3 gpurun_out/bench.err
exit $rc
