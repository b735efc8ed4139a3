set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
timeout -k 10 200 python3 tools/sweep_frame.py scenes/s_soup_1m.json '[{"shadow_ifif":0},{"shadow_ifif":1}]' 8 || exit 1
timeout -k 10 200 python3 tools/sweep_frame.py scenes/s_deep.json '[{"shadow_ifif":0},{"shadow_ifif":1}]' 8 || exit 1
done
timeout -k 10 300 python3 tools/sweep_frame.py scenes/s_soup_16m.json '[{"shadow_ifif":0},{"shadow_ifif":1},{"shadow_ifif":0}]' 2 || exit 1
