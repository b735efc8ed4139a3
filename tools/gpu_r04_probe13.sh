#!/bin/bash
# Round 4: concurrent chunks as the default: the bit-identity test, the GPU
# suite, a default bench run, and the config-5 rank frames at N = 2 / 4 / 8.
set -o pipefail
mkdir -p gpurun_out/r04e
export TMPDIR=/tmp
O=gpurun_out/r04e
timeout -k 10 700 python3 -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -rA > $O/pytest_gpu.log 2>&1
rc=$?; grep -E "concurrent_chunks|passed|failed" $O/pytest_gpu.log | tail -4; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
head -c 600 $O/bench.json; echo
for n in 2 4 8; do
  timeout -k 10 300 python3 tools/rank_pipeline.py scenes/s_deep.json $n 3 2 8 4096 > $O/pipe_sdeep4096_n${n}.jsonl 2>&1 || exit 1
  tail -n 1 $O/pipe_sdeep4096_n${n}.jsonl
done
