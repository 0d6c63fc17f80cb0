#!/bin/bash
# Sieve count kernel anatomy: kernel time per experiment mode (trace only).
set -u
S=scripts/gpu_step.sh
export TMPDIR=/tmp
B="python bench.py --config c4 --segments 1 --cpu-seconds 0 --host-gib 0 --no-tx --steps 1 --warmup 0"
for m in 0 1 2 3; do
  HVWS_SIEVE_MODE=$m $S trace_mode$m 200 rocprofv3 --kernel-trace --stats -d gpurun_out/trace_mode$m -o run --output-format csv -- $B
done
