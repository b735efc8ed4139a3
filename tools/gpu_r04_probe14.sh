#!/bin/bash
# Round 4: with concurrent chunks, does cutting a frame into more chunks pay?
# diamond N = 8 rank share (one 32 M-path chunk) at capacity 16 M / 8 M with
# two slots; diamond and S-deep frames at N = 1 with smaller chunks.
set -o pipefail
mkdir -p gpurun_out/r04f; rm -f gpurun_out/r04f/*
export TMPDIR=/tmp
O=gpurun_out/r04f
for c in 0 16000000 8000000; do
  IGX_PIPE_OPTS="{\"capacity\": $c}" timeout -k 10 200 python3 tools/rank_pipeline.py scenes/diamond_scene.json 8 8 2 >> $O/n8_capacity.jsonl 2>&1 || exit 1
done
grep '"handles": 2' $O/n8_capacity.jsonl | cut -c1-200
timeout -k 10 300 python3 tools/sweep_frame.py scenes/diamond_scene.json '[{"capacity": 0}, {"capacity": 67108864}, {"capacity": 33554432}, {"capacity": 0}, {"capacity": 67108864}]' 32 > $O/n1_capacity.log 2>&1 || exit 1
timeout -k 10 300 python3 tools/sweep_frame.py scenes/s_deep.json '[{"capacity": 0}, {"capacity": 67108864}, {"capacity": 33554432}, {"capacity": 0}, {"capacity": 67108864}]' 16 >> $O/n1_capacity.log 2>&1 || exit 1
timeout -k 10 300 python3 tools/sweep_frame.py scenes/primitives.json '[{"capacity": 0}, {"capacity": 67108864}, {"capacity": 0}, {"capacity": 67108864}]' 32 >> $O/n1_capacity.log 2>&1 || exit 1
cut -c1-110 $O/n1_capacity.log
