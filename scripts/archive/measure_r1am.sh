#!/bin/bash
set -u
S=scripts/gpu_step.sh
TAG=r1F2
export TMPDIR=/tmp
$S pytest_parity 500 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread
$S bench_$TAG 400 python bench.py
$S trace_${TAG}_c3 300 rocprofv3 --kernel-trace --stats -d gpurun_out/trace_${TAG}_c3 -o run --output-format csv -- python bench.py --steps 5 --warmup 1 --cpu-seconds 0 --host-gib 0 --no-tx
$S bench_${TAG}_c4 300 python bench.py --config c4 --segments 1024 --cpu-seconds 0 --host-gib 0 --no-tx
