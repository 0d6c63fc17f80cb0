#!/bin/bash
# Round 2: bench.py with the event-loop leg (pipelined feeder over pinned read
# buffers, 1024 connections x 20 reads, reference on one core beside it), and
# the new validation-through-feeder test.
set -u
S=scripts/gpu_step.sh
TAG=${1:-r2bb}
export TMPDIR=/tmp
rm -f gpurun_out/.stop
$S pytest_val_$TAG 300 python -u -m pytest tests/test_gpu_validate.py -x -q --timeout 120 --timeout-method thread
$S bench_$TAG 400 python3 bench.py
