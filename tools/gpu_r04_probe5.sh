#!/bin/bash
# Round 4: branch-free pushes of a 4-wide node's hit children (libigx_P.so,
# IGX_PUSH_SELECT) against the current library, interleaved twice on the
# 4-wide and quantised scenes and the diamond (fb_md5 equal = same image);
# then the 2-rank rehearsal of bench.py with the config-5 line and two stream
# slots per handle for multi-chunk shares.
set -o pipefail
mkdir -p gpurun_out/r04u
export TMPDIR=/tmp
O=gpurun_out/r04u
for round in 1 2; do for lib in libigx.so libigx_P.so; do
  export IGX_LIB_PATH=$PWD/ignis-masterthesis_amd/$lib; echo "== $lib" >> $O/ab.log
  timeout -k 10 200 python3 tools/sweep_frame.py scenes/s_deep.json '[{}]' 16 >> $O/ab.log 2>&1 || exit 1
  timeout -k 10 200 python3 tools/sweep_frame.py scenes/primitives.json '[{}]' 32 >> $O/ab.log 2>&1 || exit 1
  timeout -k 10 200 python3 tools/sweep_frame.py scenes/s_soup_1m.json '[{}]' 8 >> $O/ab.log 2>&1 || exit 1
  timeout -k 10 300 python3 tools/sweep_frame.py scenes/s_soup_16m.json '[{}]' 1 >> $O/ab.log 2>&1 || exit 1
done; done
cut -c1-170 $O/ab.log
unset IGX_LIB_PATH
export IGX_BENCH_REHEARSAL=1
timeout -k 10 500 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29502 bench.py --gpus 2 --steps 1 --warmup 1 --config5-steps 1 > $O/rehearse2.json 2> $O/rehearse2.err || { tail -5 $O/rehearse2.err; exit 1; }
grep -o '"n_gpus": [0-9]*\|"frame_equals_single_gpu": [a-z]*' $O/rehearse2.json | tr '\n' ' '; echo
