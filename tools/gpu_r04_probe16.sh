#!/bin/bash
# Round 4: asynchronous frames with igx_wait_ready at N > 1 (libigx_A.so):
# the diamond's 8-rank and 2-rank frames and config 5's 2-rank frame, two
# handles with two slots each; sequential-handle / async / async + ready;
# then the 2-rank bench rehearsal (frame check).
set -o pipefail
mkdir -p gpurun_out/r04h
export TMPDIR=/tmp
O=gpurun_out/r04h
export IGX_LIB_PATH=$PWD/ignis-masterthesis_amd/libigx_A.so
for n in 8 2; do
  for mode in "0 0" "1 0" "1 1" "0 0" "1 1"; do
    set -- $mode
    IGX_PIPE_OPTS="{\"async_render\": $1}" IGX_PIPE_READY=$2 timeout -k 10 200 python3 tools/rank_pipeline.py scenes/diamond_scene.json $n 8 2 >> $O/pipe_diamond_n$n.jsonl 2>&1 || exit 1
  done
  grep '"handles": 2' $O/pipe_diamond_n$n.jsonl | cut -c1-170
done
for mode in "0 0" "1 1"; do
  set -- $mode
  IGX_PIPE_OPTS="{\"async_render\": $1}" IGX_PIPE_READY=$2 timeout -k 10 300 python3 tools/rank_pipeline.py scenes/s_deep.json 2 3 2 8 4096 >> $O/pipe_sdeep4096_n2.jsonl 2>&1 || exit 1
done
grep '"handles": 2' $O/pipe_sdeep4096_n2.jsonl | cut -c1-170
IGX_BENCH_REHEARSAL=1 timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29502 bench.py --gpus 2 --steps 2 --warmup 1 --config5-steps 1 > $O/rehearse2.json 2> $O/rehearse2.err || { tail -5 $O/rehearse2.err; exit 1; }
grep -o '"n_gpus": [0-9]*\|"frame_equals_single_gpu": [a-z]*\|"ms_per_step": [0-9.]*' $O/rehearse2.json | tr '\n' ' '; echo
