#!/bin/bash
set -u
S=scripts/gpu_step.sh
export TMPDIR=/tmp
B="python bench.py --config c4 --segments 1 --cpu-seconds 0 --host-gib 0 --no-tx --steps 2 --warmup 1"
$S parity_sieve 400 python -u -m pytest tests/test_gpu_parity.py -x -q -k sieve --timeout 120 --timeout-method thread
$S trace3 200 rocprofv3 --kernel-trace --stats -d gpurun_out/trace3 -o run --output-format csv -- $B
