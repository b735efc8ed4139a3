#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/q_probe.py scenes/primitives.json > gpurun_out/q_prim.json 2>&1 && \
timeout -k 10 300 python3 tools/q_probe.py scenes/s_soup_1m.json > gpurun_out/q_soup.json 2>&1
rc=$?; cat gpurun_out/q_prim.json gpurun_out/q_soup.json | cut -c1-1500; exit $rc
