#!/bin/bash
set -u
S=scripts/gpu_step.sh
export TMPDIR=/tmp
$S ai_c4s_a 200 python bench.py --config c4 --segments 1 --cpu-seconds 0 --host-gib 0 --no-tx
$S ai_c4s_b 200 python bench.py --config c4 --segments 1 --cpu-seconds 0 --host-gib 0 --no-tx
$S ai_trace 300 rocprofv3 --kernel-trace --stats -d gpurun_out/trace_ai_c4s -o run --output-format csv -- python bench.py --config c4 --segments 1 --steps 4 --warmup 1 --cpu-seconds 0 --host-gib 0 --no-tx
