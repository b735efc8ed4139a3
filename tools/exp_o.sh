#!/bin/bash
# class-3 ellipsoid predicate sweep on the diamond bench frame, one rank's
# frame at N = 2, 4, 8 under several slot budgets, the shading-kind mixing
# probe, then block-regrouped shading (k_extend_rg) A/B
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/exp_o.log
: > $L
timeout -k 10 400 python3 tools/sweep_frame.py scenes/diamond_scene.json \
  '[{"class_ellipsoid_pct":0},{"class_ellipsoid_pct":100},{"class_ellipsoid_pct":85},{"class_ellipsoid_pct":70},{"class_ellipsoid_pct":115},{"class_ellipsoid_pct":0}]' 32 >> $L 2>&1 || exit 1
for n in 2 4 8; do
  timeout -k 10 300 python3 tools/rank_frame.py scenes/diamond_scene.json $n \
    '[{"slot_budget_mb":20000},{"slot_budget_mb":40000},{"slot_budget_mb":0},{"slot_budget_mb":20000}]' >> $L 2>&1 || exit 1
done
IGX_LIB_PATH=$PWD/ignis-masterthesis_amd/libigx_P.so timeout -k 10 300 python3 tools/kind_probe.py scenes/diamond_scene.json \
  '[{"path_classes":0},{"path_classes":1},{"path_classes":3},{"class_ellipsoid_pct":100},{"class_ellipsoid_pct":80,"path_classes":3}]' >> $L 2>&1 || exit 1
for sc in diamond_scene s_deep primitives; do
  it=32; [ $sc = s_deep ] && it=16
  timeout -k 10 400 python3 tools/sweep_frame.py scenes/$sc.json '[{"regroup":0},{"regroup":1},{"regroup":0},{"regroup":1}]' $it >> $L 2>&1 || exit 1
done
cut -c1-220 $L
