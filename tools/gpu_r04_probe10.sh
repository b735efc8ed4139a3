#!/bin/bash
# Round 4: the diamond's N = 8 rank frame against the tail threshold (paths at
# which a chunk's remaining paths go to the tail kernel, which overlaps the
# next frame on the other handle); auto = min(n / 64, one tail-kernel pass).
set -o pipefail
mkdir -p gpurun_out/r04z
O=gpurun_out/r04z
for t in -1 262144 524288 1048576 2097152 4194304; do
  IGX_PIPE_OPTS="{\"tail_threshold\": $t}" timeout -k 10 200 python3 tools/rank_pipeline.py scenes/diamond_scene.json 8 8 1 >> $O/tail_n8.jsonl 2>&1 || exit 1
done
grep '"handles": 2' $O/tail_n8.jsonl | cut -c1-200
for t in -1 1048576; do
  IGX_PIPE_OPTS="{\"tail_threshold\": $t}" timeout -k 10 200 python3 tools/rank_pipeline.py scenes/diamond_scene.json 1 3 2 >> $O/tail_n1.jsonl 2>&1 || exit 1
done
cut -c1-200 $O/tail_n1.jsonl
