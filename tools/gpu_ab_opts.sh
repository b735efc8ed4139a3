#!/bin/bash
# Per-scene iteration timing under several device-option sets (tools/sweep.py).
# usage: gpu_ab_opts.sh '<json list of option dicts>' scene.json ...
mkdir -p gpurun_out
OPTS="$1"; shift
for sc in "$@"; do
  echo "== $sc"
  timeout -k 10 400 python3 tools/sweep.py scenes/$sc "$OPTS" || exit 1
done
