#!/bin/bash
# A/B of a compile-time setting: per-scene iteration timing with the default
# build (A), then with the library rebuilt with EXTRA="$1" (B).
# usage: gpu_ab_build.sh "-DFOO=1" [scene ...]
mkdir -p gpurun_out
FLAGS="$1"; shift
SCENES=${@:-scenes/diamond_scene.json}
run() {
  for sc in $SCENES; do
    echo "== $1 $sc"
    timeout -k 10 400 python3 tools/sweep.py $sc '[{}]' || return 1
  done
}
run A > gpurun_out/abA.log 2>&1 || { cat gpurun_out/abA.log; exit 1; }
cat gpurun_out/abA.log
make -s -C ignis-masterthesis_amd clean >/dev/null && make -s -j16 -C ignis-masterthesis_amd EXTRA="$FLAGS" libigx.so > gpurun_out/abB_build.log 2>&1 || { cat gpurun_out/abB_build.log; exit 1; }
run "B $FLAGS" > gpurun_out/abB.log 2>&1; rc=$?
cat gpurun_out/abB.log
exit $rc
