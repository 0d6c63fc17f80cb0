#!/bin/bash
# Frame sieve: parity first, then the full GPU suite, one-stream benches, trace.
set -u
S=scripts/gpu_step.sh
TAG=${1:-r1s}
export TMPDIR=/tmp
$S pytest_sieve 300 python -u -m pytest tests/test_gpu_parity.py -k sieve -x -v --timeout 120 --timeout-method thread
$S pytest_gpu 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
$S bench_${TAG}_c4_seg1 300 python bench.py --config c4 --segments 1 --cpu-seconds 0 --host-gib 0 --no-tx --steps 5 --warmup 2
$S bench_${TAG}_c3_seg1 300 python bench.py --segments 1 --cpu-seconds 0 --host-gib 0 --no-tx --steps 5
$S bench_${TAG}_c2_seg1 300 python bench.py --config c2 --segments 1 --cpu-seconds 0 --host-gib 0 --no-tx --steps 5
$S trace_${TAG}_c4_seg1 300 rocprofv3 --kernel-trace --stats -d gpurun_out/trace_${TAG}_c4_seg1 -o run --output-format csv -- python bench.py --config c4 --segments 1 --cpu-seconds 0 --host-gib 0 --no-tx --steps 3 --warmup 1
