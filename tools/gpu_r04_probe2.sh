#!/bin/bash
# Round 4: GPU suite on the reverted layout; where a config-5 rank's frame
# goes at N = 2 (chunk of one 67 M-path iteration) against N = 1 at the same
# path count (a 2896^2 film) and with wider tiles; the per-rank frame with two
# handles alternating (bench.py's pipelining) for the diamond and config 5.
set -o pipefail
mkdir -p gpurun_out/r04q
export TMPDIR=/tmp
O=gpurun_out/r04q
timeout -k 10 600 python3 -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -rA > $O/pytest_gpu.log 2>&1
rc=$?; tail -2 $O/pytest_gpu.log; grep -E "band vs oracle|FAILED" $O/pytest_gpu.log | head -5; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/chunk_probe.py scenes/s_deep.json 1 '[{}]' 8 4096 > $O/chunk.jsonl 2>&1 || exit 1
timeout -k 10 300 python3 tools/chunk_probe.py scenes/s_deep.json 1 '[{}]' 8 2896 >> $O/chunk.jsonl 2>&1 || exit 1
timeout -k 10 300 python3 tools/chunk_probe.py scenes/s_deep.json 2 '[{}]' 8 4096 >> $O/chunk.jsonl 2>&1 || exit 1
cat $O/chunk.jsonl | cut -c1-300
for n in 2 8; do
  timeout -k 10 300 python3 tools/rank_pipeline.py scenes/diamond_scene.json $n 6 1 > $O/pipe_diamond_n$n.jsonl 2>&1 || exit 1
  timeout -k 10 300 python3 tools/rank_pipeline.py scenes/s_deep.json $n 4 1 8 4096 > $O/pipe_sdeep4096_n$n.jsonl 2>&1 || exit 1
done
tail -n 2 $O/pipe_*.jsonl
