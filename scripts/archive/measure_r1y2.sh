#!/bin/bash
# Sieve count: prefetch (mode 0) vs no prefetch (mode 4), kernel times.
set -u
S=scripts/gpu_step.sh
export TMPDIR=/tmp
B="python bench.py --config c4 --segments 1 --cpu-seconds 0 --host-gib 0 --no-tx --steps 2 --warmup 1"
for m in 0 4; do
  HVWS_SIEVE_MODE=$m $S trace_mode$m 200 rocprofv3 --kernel-trace --stats -d gpurun_out/trace2_mode$m -o run --output-format csv -- $B
done
HVWS_SIEVE_MODE=4 $S parity_mode4 400 python -u -m pytest tests/test_gpu_parity.py -x -q -k sieve --timeout 120 --timeout-method thread
