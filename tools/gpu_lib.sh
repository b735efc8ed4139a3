#!/bin/bash
# GPU job steps for gpurun, one function per step (replaces the one-off
# gpu_rNN_*.sh scripts).  Every step runs under its own time limit and
# returns its exit status, so a gpurun command chains them with &&:
#   gpurun -- 'source tools/gpu_lib.sh && gpu_tests && gpu_bench && gpu_prof'
# Output goes under gpurun_out/ (merged back by gpurun).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp

# the -m gpu suite (optionally a -k filter)
gpu_tests() {
  local k=(); [ -n "$1" ] && k=(-k "$1")
  timeout -k 10 900 python3 -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread "${k[@]}" > gpurun_out/pytest_gpu.log 2>&1
  local rc=$?; tail -3 gpurun_out/pytest_gpu.log
  [ $rc -eq 0 ] || grep -E "FAIL|Error" gpurun_out/pytest_gpu.log | head -20
  return $rc
}

# the default bench (headline + suite + CPU baseline + config-5 line); extra args pass through
gpu_bench() {
  timeout -k 10 700 python3 bench.py "$@" > gpurun_out/bench.json 2> gpurun_out/bench.err
  local rc=$?; head -c 400 gpurun_out/bench.json; echo
  [ $rc -eq 0 ] || tail -5 gpurun_out/bench.err
  return $rc
}

# rocprofv3 kernel stats of the headline (the timed frames' dispatches only)
gpu_prof() {
  rm -rf gpurun_out/prof
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- \
    python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --suite 0 --config5 0 --isolated 0 > gpurun_out/prof_bench.json 2> gpurun_out/prof.err
}

# FETCH_SIZE and WRITE_SIZE passes (one counter block each) of a scene's bench workload
# usage: gpu_pmc [iterations] [scene.json] [options json] [size] [tag]
gpu_pmc() {
  local it=${1:-32} sc=${2:-diamond_scene.json} op=${3:-'{}'} sz=${4:-0} tag=${5:-headline}
  rm -rf gpurun_out/pmc_${tag}_fetch gpurun_out/pmc_${tag}_write
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_${tag}_fetch -o run --output-format csv -- \
    python3 tools/pmc_run.py $it $sc "$op" $sz > gpurun_out/pmc_${tag}_fetch.log 2>&1 && \
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_${tag}_write -o run --output-format csv -- \
    python3 tools/pmc_run.py $it $sc "$op" $sz > gpurun_out/pmc_${tag}_write.log 2>&1
}

# rocprof + PMC evidence of the suite lines (tools/gpu_profile_suite.sh keys)
gpu_suite_prof() {
  bash tools/gpu_profile_suite.sh "$@"
}

# one bench frame of a scene under option sets: gpu_frame scene.json iterations '[{...}, ...]' [WxH]
gpu_frame() {
  local sc=$1 it=$2 op=${3:-'[{}]'} sz=$4
  timeout -k 10 400 python3 tools/sweep_frame.py scenes/$sc "$op" $it $sz 2>&1 | tee -a gpurun_out/frames.log
}

# library A/B (tools/ab_libs.sh): gpu_ab "libigx.so libigx_X.so" scenes/a.json ...
gpu_ab() {
  local libs=$1; shift
  bash tools/ab_libs.sh "$libs" "$@" 2>&1 | tee -a gpurun_out/ab.log
}

# instrumented traversal statistics of one iteration: gpu_stats scene.json [options json]
gpu_stats() {
  local op=$2; [ -n "$op" ] || op='{}'
  timeout -k 10 300 python3 tools/ray_stats.py scenes/$1 "$op" 2>&1 | tee -a gpurun_out/ray_stats.log
}

# the launcher's N-rank rehearsal on one GPU (gloo, every rank on GPU 0)
gpu_rehearse() {
  local n=${1:-2}
  IGX_BENCH_REHEARSAL=1 timeout -k 10 600 python3 bench.py --gpus $n --steps 2 --warmup 1 --config5-steps 1 \
    > gpurun_out/rehearse$n.json 2> gpurun_out/rehearse$n.err
  local rc=$?; grep -o '"frame_equals_single_gpu": [a-z]*' gpurun_out/rehearse$n.json | tr '\n' ' '; echo
  [ $rc -eq 0 ] || tail -5 gpurun_out/rehearse$n.err
  return $rc
}

# kernel trace of an arbitrary python tool: gpu_trace tag tools/x.py args...
gpu_trace() {
  local tag=$1; shift
  rm -rf gpurun_out/trace_$tag
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/trace_$tag -o run --output-format csv -- \
    python3 "$@" > gpurun_out/trace_$tag.log 2>&1
}

# round-6 SQ / L2 / LDS counter passes: gpu_sq TAG ITERATIONS SCENE [OPTIONS_JSON] [SIZE]
gpu_sq() {
  bash tools/gpu_pmc_sq.sh "$@" && python3 tools/pmc_sq_summary.py gpurun_out/sq_$1 gpurun_out/sq_$1.json
}

# rank frames of the N-GPU shares on one GPU (tools/rank_pipeline.py, two
# handles alternating as bench.py does at N > 1): gpu_ranks TAG SCENE ITERATIONS SIZE "N..." [stream_slots]
gpu_ranks() {
  local tag=$1 sc=$2 it=$3 sz=$4 ns=$5 slots=${6:-1}
  for n in $ns; do
    echo "== $tag n$n" | tee -a gpurun_out/ranks_$tag.log
    IGX_PIPE_READY=1 timeout -k 10 300 python3 tools/rank_pipeline.py scenes/$sc $n 6 $slots $it $sz 2>&1 | tee -a gpurun_out/ranks_$tag.log || return 1
  done
}
