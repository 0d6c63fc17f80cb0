#!/bin/bash
# SLACK table: parity file, c4 (1024 connections), c2, c3.
set -u
S=scripts/gpu_step.sh
TAG=${1:-r1ac}
export TMPDIR=/tmp
$S pytest_parity 500 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread
$S bench_${TAG}_c4 300 python bench.py --config c4 --segments 1024 --cpu-seconds 0 --host-gib 0 --no-tx
$S bench_${TAG}_c2 300 python bench.py --config c2 --cpu-seconds 0 --host-gib 0 --no-tx
$S bench_${TAG}_c3 300 python bench.py --cpu-seconds 0 --host-gib 0 --no-tx
$S trace_${TAG}_c4 300 rocprofv3 --kernel-trace --stats -d gpurun_out/trace_${TAG}_c4 -o run --output-format csv -- python bench.py --config c4 --segments 1024 --steps 4 --warmup 1 --cpu-seconds 0 --host-gib 0 --no-tx
