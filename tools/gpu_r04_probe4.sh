#!/bin/bash
# Round 4: S-deep with quantised 4-wide nodes (now with the octant-ordered
# quantised slab test) against 128-B float nodes, interleaved; then where a
# config-5 rank's frame goes at N = 2 against N = 1 at the same path count
# (2896^2 film), and the per-rank frame with two handles alternating (bench.py's
# pipelining) for the diamond and config 5.
set -o pipefail
mkdir -p gpurun_out/r04t
export TMPDIR=/tmp
O=gpurun_out/r04t
for round in 1 2; do
  timeout -k 10 240 python3 tools/sweep_frame.py scenes/s_deep.json '[{}, {"bvh_quantize": 1}, {"bvh_quantize": 0}]' 16 >> $O/ab_q4.log 2>&1 || exit 1
done
cut -c1-200 $O/ab_q4.log
timeout -k 10 300 python3 tools/chunk_probe.py scenes/s_deep.json 1 '[{}]' 8 4096 > $O/chunk.jsonl 2>&1 || exit 1
timeout -k 10 300 python3 tools/chunk_probe.py scenes/s_deep.json 1 '[{}]' 8 2896 >> $O/chunk.jsonl 2>&1 || exit 1
timeout -k 10 300 python3 tools/chunk_probe.py scenes/s_deep.json 2 '[{}]' 8 4096 >> $O/chunk.jsonl 2>&1 || exit 1
cut -c1-300 $O/chunk.jsonl
for n in 2 8; do
  timeout -k 10 300 python3 tools/rank_pipeline.py scenes/diamond_scene.json $n 6 1 > $O/pipe_diamond_n$n.jsonl 2>&1 || exit 1
  timeout -k 10 300 python3 tools/rank_pipeline.py scenes/s_deep.json $n 4 1 8 4096 > $O/pipe_sdeep4096_n$n.jsonl 2>&1 || exit 1
done
tail -n 2 $O/pipe_*.jsonl | cut -c1-400
