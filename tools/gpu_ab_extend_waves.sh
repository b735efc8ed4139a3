set -o pipefail
for round in 1 2; do for lib in libigx.so libigx_B.so; do
  export IGX_LIB_PATH=$PWD/ignis-masterthesis_amd/$lib; echo "== $lib"
  timeout -k 10 200 python3 tools/sweep_frame.py scenes/s_deep.json '[{}]' 8 || exit 1
  timeout -k 10 200 python3 tools/sweep_frame.py scenes/primitives.json '[{}]' 32 || exit 1
  timeout -k 10 200 python3 tools/sweep_frame.py scenes/materials.json '[{}]' 32 || exit 1
done; done
