#!/bin/bash
# One-GPU dry run of bench.py's multi-GPU path: N ranks (torch.distributed.run)
# share GPU 0 over gloo with host staging (IGX_BENCH_REHEARSAL=1) and rank 0
# checks the gathered tile-sharded frame equals a single-device render bit for bit.
# usage: gpu_rehearse_multi.sh [N ...]   (default 2 4)
mkdir -p gpurun_out
export IGX_BENCH_REHEARSAL=1
for n in ${@:-2 4}; do
  timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $((29500 + n)) bench.py --gpus $n --steps 2 --warmup 1 --check-frame \
    > gpurun_out/rehearse$n.json 2> gpurun_out/rehearse$n.err || { tail -5 gpurun_out/rehearse$n.err; exit 1; }
  grep -o '"n_gpus": [0-9]*\|"frame_equals_single_gpu": [a-z]*' gpurun_out/rehearse$n.json | tr '\n' ' '; echo
  grep -q '"frame_equals_single_gpu": true' gpurun_out/rehearse$n.json || exit 1
done
