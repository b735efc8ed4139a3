#!/bin/bash
# Round 4 probes: config-5 rank shares by chunk capacity / slots (where the
# N = 2 share loses time), and S-deep 1000^2 k_extend levers (quantised
# nodes, split schedule, 5 waves per SIMD build).
set -o pipefail
mkdir -p gpurun_out/r04p
export TMPDIR=/tmp
O=gpurun_out/r04p
timeout -k 10 300 python3 tools/chunk_probe.py scenes/s_deep.json 1 '[{}, {"capacity": 67108864}]' > $O/chunk_n1.jsonl 2>&1 || exit 1
timeout -k 10 300 python3 tools/chunk_probe.py scenes/s_deep.json 2 '[{}, {"capacity": 33554432}, {"capacity": 0, "stream_slots": 1}]' > $O/chunk_n2.jsonl 2>&1 || exit 1
timeout -k 10 300 python3 tools/chunk_probe.py scenes/s_deep.json 4 '[{}]' > $O/chunk_n4.jsonl 2>&1 || exit 1
cat $O/chunk_n*.jsonl
for round in 1 2; do
  timeout -k 10 300 python3 tools/sweep_frame.py scenes/s_deep.json '[{}, {"split": 1}, {"split": -1, "bvh_quantize": 1}]' 16 >> $O/sdeep_opts.jsonl 2>&1 || exit 1
  IGX_LIB_PATH=$PWD/ignis-masterthesis_amd/libigx_W.so timeout -k 10 300 python3 tools/sweep_frame.py scenes/s_deep.json '[{}]' 16 >> $O/sdeep_w5.jsonl 2>&1 || exit 1
done
cat $O/sdeep_opts.jsonl $O/sdeep_w5.jsonl
