#!/bin/bash
# Round 2: default bench with the event-loop leg taking the median of 3 passes.
set -u
S=scripts/gpu_step.sh
TAG=${1:-r2bs}
export TMPDIR=/tmp
rm -f gpurun_out/.stop
$S bench_$TAG 400 python3 bench.py
