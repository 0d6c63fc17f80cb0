#!/bin/bash
# Round 2: GPU suite + smoke + default bench on the current tree (k_small
# staged in LDS, zero-copy small batches, host copy pool).
set -u
S=scripts/gpu_step.sh
TAG=${1:-r2ap}
export TMPDIR=/tmp
rm -f gpurun_out/.stop
$S pytest_gpu_$TAG 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
$S smoke_$TAG 120 python3 -c "import __graft_entry__ as g; g.smoke()"
$S bench_$TAG 300 python3 bench.py
