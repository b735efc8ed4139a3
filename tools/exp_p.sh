#!/bin/bash
# three path classes (class C region) vs two on the bench frame; one vs two
# stream slots per handle on a rank's frame (two handles alternating,
# bench.py's N > 1 pipeline); the GPU tests of both
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/exp_p.log
: > $L
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu.py -k "one_stream_slot or render_iterations_equals or path_class" >> $L 2>&1 || { tail -30 $L; exit 1; }
timeout -k 10 400 python3 tools/sweep_frame.py scenes/diamond_scene.json '[{"path_classes":3},{"path_classes":4},{"path_classes":3},{"path_classes":4}]' 32 >> $L 2>&1 || exit 1
for sc in s_deep primitives; do
  timeout -k 10 400 python3 tools/sweep_frame.py scenes/$sc.json '[{"path_classes":3},{"path_classes":4},{"path_classes":3},{"path_classes":4}]' 16 >> $L 2>&1 || exit 1
done
for n in 2 8; do
  for sl in 2 1; do
    timeout -k 10 300 python3 tools/rank_pipeline.py scenes/diamond_scene.json $n 6 $sl >> $L 2>&1 || exit 1
  done
done
cat $L | cut -c1-220
