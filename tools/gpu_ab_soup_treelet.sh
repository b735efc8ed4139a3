set -o pipefail
mkdir -p gpurun_out
for round in 1 2; do for lib in libigx.so libigx_X.so; do
  export IGX_LIB_PATH=$PWD/ignis-masterthesis_amd/$lib; echo "== $lib"
  timeout -k 10 200 python3 tools/sweep_frame.py scenes/s_soup_1m.json '[{},{"treelet_kernels":7}]' 8 || exit 1
  if [ $round = 1 ]; then timeout -k 10 300 python3 tools/sweep_frame.py scenes/s_soup_16m.json '[{},{"treelet_kernels":7}]' 2 || exit 1; fi
done; done
