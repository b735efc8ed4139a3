#!/bin/bash
# Round 4: async frames with one stream slot per handle (libigx_A.so):
# targeted GPU tests, the diamond's 8-rank and 2-rank frames (sync / async +
# igx_wait_ready), the 2-rank bench rehearsal (frame check), the GPU suite.
set -o pipefail
mkdir -p gpurun_out/r04i
export TMPDIR=/tmp
O=gpurun_out/r04i
export IGX_LIB_PATH=$PWD/ignis-masterthesis_amd/libigx_A.so
timeout -k 10 300 python3 -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread -k "concurrent_chunks or async_render or shard or pack" > $O/pytest_new.log 2>&1
rc=$?; tail -2 $O/pytest_new.log; [ $rc -eq 0 ] || exit $rc
for n in 8 2; do
  for mode in "0 0" "1 1" "0 0" "1 1"; do
    set -- $mode
    IGX_PIPE_OPTS="{\"async_render\": $1}" IGX_PIPE_READY=$2 timeout -k 10 200 python3 tools/rank_pipeline.py scenes/diamond_scene.json $n 8 1 >> $O/pipe_diamond_n$n.jsonl 2>&1 || exit 1
  done
  grep '"handles": 2' $O/pipe_diamond_n$n.jsonl | cut -c1-170
done
IGX_BENCH_REHEARSAL=1 timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29502 bench.py --gpus 2 --steps 2 --warmup 1 --config5-steps 1 > $O/rehearse2.json 2> $O/rehearse2.err || { tail -5 $O/rehearse2.err; exit 1; }
grep -o '"n_gpus": [0-9]*\|"frame_equals_single_gpu": [a-z]*\|"ms_per_step": [0-9.]*' $O/rehearse2.json | tr '\n' ' '; echo
timeout -k 10 700 python3 -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -2 $O/pytest_gpu.log; exit $rc
