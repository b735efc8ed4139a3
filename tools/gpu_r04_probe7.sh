#!/bin/bash
# Round 4: kernel timelines (rocprofv3 --kernel-trace) of one config-5 rank
# frame at N = 2 (4096^2 tile share, two stream slots) and of a 2896^2 film
# with the same path count at N = 1, to find where the rank's frame idles.
set -o pipefail
mkdir -p gpurun_out/r04w
export TMPDIR=/tmp
O=gpurun_out/r04w
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/n2 -o run --output-format csv -- python3 tools/chunk_probe.py scenes/s_deep.json 2 '[{"stream_slots": 2}]' 8 4096 > $O/n2.log 2>&1 || { tail -5 $O/n2.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/n1 -o run --output-format csv -- python3 tools/chunk_probe.py scenes/s_deep.json 1 '[{"stream_slots": 2}]' 8 2896 > $O/n1.log 2>&1 || { tail -5 $O/n1.log; exit 1; }
grep '^{' $O/n2.log $O/n1.log | cut -c1-300
find $O -name "*kernel_trace.csv" | head
