#!/bin/bash
# Round 4: bench.py's config-5 line and per-rank breakdown on one GPU (N = 1,
# and the N = 2 rehearsal through bench.py's own launcher: both ranks on GPU 0
# over gloo), then the simulated strong scaling of the diamond (config 2) and
# of S-deep 4096^2 64 spp (config 5) with the current kernels.
set -o pipefail
mkdir -p gpurun_out/r04m
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --suite 0 --no-cpu-baseline > gpurun_out/r04m/bench_n1.json 2> gpurun_out/r04m/bench_n1.err || { tail -5 gpurun_out/r04m/bench_n1.err; exit 1; }
head -c 300 gpurun_out/r04m/bench_n1.json; echo
IGX_BENCH_REHEARSAL=1 timeout -k 10 400 python3 bench.py --gpus 2 --steps 2 --warmup 1 > gpurun_out/r04m/rehearse2.json 2> gpurun_out/r04m/rehearse2.err || { tail -5 gpurun_out/r04m/rehearse2.err; exit 1; }
grep -o '"frame_equals_single_gpu": [a-z]*' gpurun_out/r04m/rehearse2.json | tr '\n' ' '; echo
timeout -k 10 300 python3 tools/shard_sim.py scenes/diamond_scene.json > gpurun_out/r04m/shard_sim_diamond.jsonl 2>&1 || exit 1
timeout -k 10 400 python3 tools/shard_sim.py scenes/s_deep.json 0 4096x4096 8 > gpurun_out/r04m/shard_sim_s_deep_4096.jsonl 2>&1 || exit 1
cat gpurun_out/r04m/shard_sim_*.jsonl
