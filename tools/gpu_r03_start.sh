#!/bin/bash
# Round-3 first GPU session: host CPU facts, GPU tests, the default bench, a
# bench.py --gpus 2 rehearsal through the new launcher, and the suite profiles.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
{ nproc; python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)), 'cpu_count', os.cpu_count(), 'omp', os.environ.get('OMP_NUM_THREADS'))"; cat /sys/fs/cgroup/cpu.max 2>/dev/null; cat /proc/self/status | grep -i cpus_allowed_list; } > gpurun_out/cpuinfo.txt 2>&1
cat gpurun_out/cpuinfo.txt
timeout -k 10 600 python3 -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err && cat gpurun_out/bench.json | head -c 1500 && echo && \
IGX_BENCH_REHEARSAL=1 timeout -k 10 400 python3 bench.py --gpus 2 --steps 2 --warmup 1 --check-frame > gpurun_out/rehearse2.json 2> gpurun_out/rehearse2.err && \
grep -o '"n_gpus": [0-9]*\|"frame_equals_single_gpu": [a-z]*\|"slot_bytes_per_handle": [^]]*]\|"backend": "[^"]*"' gpurun_out/rehearse2.json && \
bash tools/gpu_profile_suite.sh
rc=$?
echo "rc=$rc"
exit $rc
