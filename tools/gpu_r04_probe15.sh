#!/bin/bash
# Round 4: asynchronous rendering (libigx_A.so, option async_render): the
# bit-identity tests, the GPU suite, bench at N = 1 (async on / off), the
# diamond's N = 8 and N = 1 rank frames and config 5's at N = 2.
set -o pipefail
mkdir -p gpurun_out/r04g
export TMPDIR=/tmp
O=gpurun_out/r04g
export IGX_LIB_PATH=$PWD/ignis-masterthesis_amd/libigx_A.so
timeout -k 10 300 python3 -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread -k "concurrent_chunks or async_render" > $O/pytest_new.log 2>&1
rc=$?; tail -3 $O/pytest_new.log; [ $rc -eq 0 ] || exit $rc
for a in 0 1 0 1; do
  IGX_PIPE_OPTS="{\"async_render\": $a}" timeout -k 10 200 python3 tools/rank_pipeline.py scenes/diamond_scene.json 8 8 1 >> $O/pipe_diamond_n8.jsonl 2>&1 || exit 1
done
grep '"handles": 2' $O/pipe_diamond_n8.jsonl | cut -c1-160
for a in 0 1; do
  IGX_PIPE_OPTS="{\"async_render\": $a}" timeout -k 10 300 python3 tools/rank_pipeline.py scenes/diamond_scene.json 1 4 2 >> $O/pipe_diamond_n1.jsonl 2>&1 || exit 1
  IGX_PIPE_OPTS="{\"async_render\": $a}" timeout -k 10 300 python3 tools/rank_pipeline.py scenes/s_deep.json 2 3 2 8 4096 >> $O/pipe_sdeep4096_n2.jsonl 2>&1 || exit 1
done
cut -c1-160 $O/pipe_diamond_n1.jsonl $O/pipe_sdeep4096_n2.jsonl
timeout -k 10 600 python3 bench.py --suite 0 --no-cpu-baseline --config5 0 > $O/bench_async.json 2> $O/bench_async.err || { tail -5 $O/bench_async.err; exit 1; }
head -c 300 $O/bench_async.json; echo
timeout -k 10 700 python3 -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; exit $rc
