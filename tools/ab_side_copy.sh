set -o pipefail
for r in 1 2; do for lib in libigx.so libigx_nocopy.so; do
  echo "== $lib"
  IGX_LIB_PATH=$PWD/ignis-masterthesis_amd/$lib timeout -k 10 300 python3 tools/sweep_frame.py scenes/diamond_scene.json '[{}]' 32 || exit 1
  IGX_LIB_PATH=$PWD/ignis-masterthesis_amd/$lib timeout -k 10 300 python3 tools/sweep_frame.py scenes/s_deep.json '[{}]' 32 || exit 1
  IGX_LIB_PATH=$PWD/ignis-masterthesis_amd/$lib IGX_PIPE_READY=1 timeout -k 10 300 python3 tools/rank_pipeline.py scenes/diamond_scene.json 8 6 1 32 || exit 1
done; done
