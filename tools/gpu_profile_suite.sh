#!/bin/bash
# rocprofv3 evidence for every suite line of bench.py (SURVEY.md §8d configs
# 3-5 and the soups): per scene one --kernel-trace --stats pass and separate
# FETCH_SIZE / WRITE_SIZE counter passes over the suite's own workload
# (tools/pmc_run.py: same scene, film and iteration count as the suite line).
# tools/profile_summary.py suite <tag> turns them into profiles/.
# usage: gpu_profile_suite.sh [key ...]   (default: all)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
declare -A ITERS=([primitives]=8 [s_deep]=128 [s_soup_1m]=2 [s_soup_16m]=1 [s_deep_4096]=8)
declare -A SCENE=([primitives]=primitives.json [s_deep]=s_deep.json [s_soup_1m]=s_soup_1m.json [s_soup_16m]=s_soup_16m.json [s_deep_4096]=s_deep.json)
declare -A SIZE=([primitives]=0 [s_deep]=0 [s_soup_1m]=0 [s_soup_16m]=0 [s_deep_4096]=4096)
# split-schedule scenes: the trace kernel alone (overlap_shadow 0), the
# duration bench.py's roofline["isolated"] reports next to this profile
declare -A OPTS=([primitives]='{}' [s_deep]='{}' [s_soup_1m]='{"overlap_shadow":0}' [s_soup_16m]='{"overlap_shadow":0}' [s_deep_4096]='{}')
rm -f gpurun_out/suite.log
for key in ${@:-primitives s_deep s_deep_4096 s_soup_1m s_soup_16m}; do
  d=gpurun_out/suite_$key
  rm -rf $d && mkdir -p $d
  args="${ITERS[$key]} ${SCENE[$key]} ${OPTS[$key]} ${SIZE[$key]}"
  echo "== $key: pmc_run.py $args" | tee -a gpurun_out/suite.log
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $d/trace -o run --output-format csv -- python3 tools/pmc_run.py $args > $d/trace.log 2>&1 || { tail -5 $d/trace.log; exit 1; }
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $d/fetch -o run --output-format csv -- python3 tools/pmc_run.py $args > $d/fetch.log 2>&1 || { tail -5 $d/fetch.log; exit 1; }
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $d/write -o run --output-format csv -- python3 tools/pmc_run.py $args > $d/write.log 2>&1 || { tail -5 $d/write.log; exit 1; }
done
echo "suite profiles done"
