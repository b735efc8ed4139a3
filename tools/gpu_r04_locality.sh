#!/bin/bash
# Round 4: full GPU suite on the screen-local generation layout, then A/B of
# gen_layout 0 (round-robin groups) / 1 (one film band per XCD) per scene,
# interleaved twice (tools/sweep_frame.py: best of 2 reps, fb_md5 = image)
set -o pipefail
mkdir -p gpurun_out/r04l
export TMPDIR=/tmp
O=gpurun_out/r04l
timeout -k 10 600 python3 -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -rA ${PYTEST_K:+-k "$PYTEST_K"} > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; grep -E "halves RelSE|band vs oracle|FAILED|Error" $O/pytest_gpu.log | head -5; [ $rc -eq 0 ] || exit $rc
for round in 1 2; do
  timeout -k 10 200 python3 tools/sweep_frame.py scenes/s_soup_16m.json '[{"gen_layout":0},{"gen_layout":1}]' 1 >> $O/ab_soup16m.jsonl 2>&1 || exit 1
  timeout -k 10 200 python3 tools/sweep_frame.py scenes/s_soup_1m.json '[{"gen_layout":0},{"gen_layout":1}]' 2 >> $O/ab_soup1m.jsonl 2>&1 || exit 1
  timeout -k 10 200 python3 tools/sweep_frame.py scenes/s_deep.json '[{"gen_layout":0},{"gen_layout":1}]' 16 >> $O/ab_sdeep.jsonl 2>&1 || exit 1
  timeout -k 10 200 python3 tools/sweep_frame.py scenes/diamond_scene.json '[{"gen_layout":0},{"gen_layout":1}]' 32 >> $O/ab_diamond.jsonl 2>&1 || exit 1
  timeout -k 10 200 python3 tools/sweep_frame.py scenes/primitives.json '[{"gen_layout":0},{"gen_layout":1}]' 8 >> $O/ab_primitives.jsonl 2>&1 || exit 1
done
for f in $O/ab_*.jsonl; do echo "== $f"; cut -c1-200 $f; done
