#!/bin/bash
# Round-1 (session e) pass: GPU tests, bench (c3, c2), per-dispatch kernel
# traces of both for the step-gap analysis (scripts/trace_gaps.py).
set -u
S=scripts/gpu_step.sh
TAG=${1:-r1e}
export TMPDIR=/tmp
$S pytest_gpu 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
$S bench_$TAG 400 python bench.py
$S bench_${TAG}_c2 300 python bench.py --config c2 --cpu-seconds 2 --host-gib 1
$S trace_${TAG}_c3 300 rocprofv3 --kernel-trace --stats -d gpurun_out/trace_${TAG}_c3 -o run --output-format csv -- python bench.py --steps 5 --warmup 1 --cpu-seconds 0 --host-gib 0 --no-tx
$S trace_${TAG}_c2 300 rocprofv3 --kernel-trace --stats -d gpurun_out/trace_${TAG}_c2 -o run --output-format csv -- python bench.py --config c2 --steps 5 --warmup 1 --cpu-seconds 0 --host-gib 0 --no-tx
