#!/bin/bash
# Round 4: the default 1-GPU bench (headline + suite + config-5 line) and the
# launcher's 2- and 4-rank rehearsals on one GPU (IGX_BENCH_REHEARSAL=1: gloo,
# every rank on GPU 0) with the config-5 line's pre-flight and frame check.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 bench.py > gpurun_out/bench1.json 2> gpurun_out/bench1.err || { tail -5 gpurun_out/bench1.err; exit 1; }
head -c 300 gpurun_out/bench1.json; echo
for n in 2 4; do
  IGX_BENCH_REHEARSAL=1 timeout -k 10 500 python3 bench.py --gpus $n --steps 2 --warmup 1 --config5-steps 1 > gpurun_out/rehearse$n.json 2> gpurun_out/rehearse$n.err || { tail -5 gpurun_out/rehearse$n.err; exit 1; }
  echo "n=$n done"
done
