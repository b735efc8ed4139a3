#!/bin/bash
# Round 4: per-rank frame of config 5 (S-deep 4096^2, 8 iterations) with two
# stream slots per handle (bench.py rank_stream_slots) at N = 2 / 4 / 8, two
# handles alternating; and where the diamond's N = 8 rank frame goes (its tile
# share against a 354^2 film of the same path count).
set -o pipefail
mkdir -p gpurun_out/r04v
export TMPDIR=/tmp
O=gpurun_out/r04v
for n in 2 4 8; do
  timeout -k 10 300 python3 tools/rank_pipeline.py scenes/s_deep.json $n 3 2 8 4096 > $O/pipe_sdeep4096_n${n}_slots2.jsonl 2>&1 || exit 1
  tail -n 1 $O/pipe_sdeep4096_n${n}_slots2.jsonl
done
timeout -k 10 300 python3 tools/chunk_probe.py scenes/diamond_scene.json 8 '[{"stream_slots": 1}, {"stream_slots": 2}]' 32 1000 > $O/chunk_diamond.jsonl 2>&1 || exit 1
timeout -k 10 300 python3 tools/chunk_probe.py scenes/diamond_scene.json 1 '[{"stream_slots": 1}, {"stream_slots": 2}]' 32 354 >> $O/chunk_diamond.jsonl 2>&1 || exit 1
cut -c1-400 $O/chunk_diamond.jsonl
