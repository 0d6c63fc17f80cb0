#!/bin/bash
set -u
S=scripts/gpu_step.sh
export TMPDIR=/tmp
$S trace_c4 300 rocprofv3 --kernel-trace --stats -d gpurun_out/trace_ab_c4 -o run --output-format csv -- python bench.py --config c4 --segments 1024 --steps 4 --warmup 1 --cpu-seconds 0 --host-gib 0 --no-tx
$S trace_c4s 300 rocprofv3 --kernel-trace --stats -d gpurun_out/trace_ab_c4s -o run --output-format csv -- python bench.py --config c4 --segments 1024 --steps 4 --warmup 1 --cpu-seconds 0 --host-gib 0 --no-tx --serial
