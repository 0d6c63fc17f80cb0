#!/bin/bash
# Round 2: unmask geometry chosen by batch size.  GPU suite (incl. every
# geometry on every tile class), then the default bench at c2, c4 and c3.
set -u
S=scripts/gpu_step.sh
TAG=${1:-r2m}
export TMPDIR=/tmp
rm -f gpurun_out/.stop
$S pytest_gpu_$TAG 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
B="python3 bench.py --cpu-seconds 0 --host-gib 0 --no-tx"
$S bench_${TAG}_c2 200 $B --steps 200 --warmup 10 --config c2
$S bench_${TAG}_c4 200 $B --steps 100 --warmup 10 --config c4 --segments 1024
$S bench_${TAG}_c4_seg1 300 $B --steps 20 --warmup 5 --config c4 --segments 1
$S bench_${TAG}_c3 400 python3 bench.py
