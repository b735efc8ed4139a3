set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/sweep_frame.py scenes/diamond_scene.json '[{"path_classes":1},{"path_classes":3},{"path_classes":1},{"path_classes":3},{"path_classes":0}]' 32 > gpurun_out/exp1_diamond.log 2>&1 && \
timeout -k 10 300 python3 tools/sweep_frame.py scenes/materials.json '[{"path_classes":1},{"path_classes":3},{"path_classes":1},{"path_classes":3}]' 32 > gpurun_out/exp1_materials.log 2>&1
rc=$?; cat gpurun_out/exp1_*.log; exit $rc
