#!/bin/bash
# Frame sieve iteration: sieve parity, per-step diagnostic, one-stream c4 bench + trace.
set -u
S=scripts/gpu_step.sh
TAG=${1:-r1t}
export TMPDIR=/tmp
$S pytest_parity 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread
$S debug_sieve 200 python scripts/debug_sieve.py
$S bench_${TAG}_c4_seg1 300 python bench.py --config c4 --segments 1 --cpu-seconds 0 --host-gib 0 --no-tx --steps 5 --warmup 2
$S trace_${TAG}_c4_seg1 300 rocprofv3 --kernel-trace --stats -d gpurun_out/trace_${TAG}_c4_seg1 -o run --output-format csv -- python bench.py --config c4 --segments 1 --cpu-seconds 0 --host-gib 0 --no-tx --steps 3 --warmup 1
