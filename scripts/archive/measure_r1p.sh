#!/bin/bash
# GPU tests, bench c3/c2, one-stream c3/c4, host-inclusive chunk sizes.
set -u
S=scripts/gpu_step.sh
TAG=${1:-r1p}
export TMPDIR=/tmp
$S pytest_gpu 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
$S bench_$TAG 400 python bench.py
$S bench_${TAG}_c2 300 python bench.py --config c2 --cpu-seconds 2 --host-gib 1
$S bench_${TAG}_c3_seg1 300 python bench.py --segments 1 --cpu-seconds 0 --host-gib 0 --no-tx --steps 5
$S bench_${TAG}_c4_seg1 300 python bench.py --config c4 --segments 1 --cpu-seconds 0 --host-gib 0 --no-tx --steps 3 --warmup 1
$S bench_${TAG}_c3_chunk64 300 python bench.py --cpu-seconds 0 --host-chunk-mib 64 --no-tx --steps 3
