#!/bin/bash
# Round 4: concurrent chunks with a staggered start (option
# concurrent_start_pct: the next chunk starts once the running one is down to
# that share of its paths) against the sequential schedule; and frames on
# worker threads over two handles (tools/rank_pipeline.py IGX_PIPE_THREADS).
set -o pipefail
mkdir -p gpurun_out/r04d
export TMPDIR=/tmp
O=gpurun_out/r04d
export IGX_LIB_PATH=$PWD/ignis-masterthesis_amd/libigx_C.so
AB='[{"concurrent_chunks": 0}, {"concurrent_chunks": 1, "concurrent_start_pct": 5}, {"concurrent_start_pct": 10}, {"concurrent_start_pct": 25}, {"concurrent_start_pct": 100}, {"concurrent_chunks": 0}, {"concurrent_chunks": 1, "concurrent_start_pct": 5}, {"concurrent_start_pct": 10}, {"concurrent_start_pct": 25}]'
timeout -k 10 300 python3 tools/sweep_frame.py scenes/diamond_scene.json "$AB" 32 > $O/ab.log 2>&1 || { tail -5 $O/ab.log; exit 1; }
timeout -k 10 300 python3 tools/sweep_frame.py scenes/primitives.json "$AB" 32 >> $O/ab.log 2>&1 || { tail -5 $O/ab.log; exit 1; }
timeout -k 10 500 python3 tools/sweep_frame.py scenes/s_deep.json "$AB" 8 4096x4096 >> $O/ab.log 2>&1 || { tail -5 $O/ab.log; exit 1; }
cut -c1-120 $O/ab.log
for n in 8 1; do
  IGX_PIPE_THREADS=1 timeout -k 10 300 python3 tools/rank_pipeline.py scenes/diamond_scene.json $n 8 $([ $n = 8 ] && echo 1 || echo 2) > $O/threads_diamond_n$n.jsonl 2>&1 || { tail -5 $O/threads_diamond_n$n.jsonl; exit 1; }
  cat $O/threads_diamond_n$n.jsonl
done
