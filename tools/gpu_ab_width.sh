#!/bin/bash
# GPU tests, then per-scene iteration timing with BVH width auto / 2 / 4.
mkdir -p gpurun_out
timeout -k 10 400 python3 -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -4 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
OPTS=${1:-'[{"bvh_width": 0}, {"bvh_width": 2}, {"bvh_width": 4}]'}
for sc in scenes/diamond_scene.json scenes/primitives.json scenes/s_deep.json scenes/s_soup_1m.json scenes/s_soup_16m.json; do
  echo "== $sc"
  timeout -k 10 400 python3 tools/sweep.py $sc "$OPTS" || exit 1
done > gpurun_out/ab.log 2>&1; rc=$?
cat gpurun_out/ab.log
exit $rc
