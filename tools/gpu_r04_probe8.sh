#!/bin/bash
# Round 4: after the closed-form valid_pixels_in_chunk: tile-shard GPU tests,
# the config-5 rank frame (two slots, two handles) at N = 2 / 4 / 8, the
# diamond's at N = 2 / 8, and the N = 2 rank's kernel timeline again.
set -o pipefail
mkdir -p gpurun_out/r04x
export TMPDIR=/tmp
O=gpurun_out/r04x
timeout -k 10 400 python3 -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -k "config5 or shard or counters or pack or config4" > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for n in 2 4 8; do
  timeout -k 10 300 python3 tools/rank_pipeline.py scenes/s_deep.json $n 3 2 8 4096 > $O/pipe_sdeep4096_n${n}.jsonl 2>&1 || exit 1
  tail -n 1 $O/pipe_sdeep4096_n${n}.jsonl
done
for n in 2 8; do
  timeout -k 10 300 python3 tools/rank_pipeline.py scenes/diamond_scene.json $n 6 1 > $O/pipe_diamond_n$n.jsonl 2>&1 || exit 1
  tail -n 1 $O/pipe_diamond_n$n.jsonl
done
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/n2 -o run --output-format csv -- python3 tools/chunk_probe.py scenes/s_deep.json 2 '[{"stream_slots": 2}]' 8 4096 > $O/n2.log 2>&1 || { tail -5 $O/n2.log; exit 1; }
grep '^{' $O/n2.log | cut -c1-300
