#!/bin/bash
# Round 2, last call of the session: the driver's round-end commands on the
# final tree (GPU suite, smoke, default bench).
set -u
S=scripts/gpu_step.sh
TAG=${1:-r2bp}
export TMPDIR=/tmp
rm -f gpurun_out/.stop
$S pytest_gpu_$TAG 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
$S smoke_$TAG 120 python3 -c "import __graft_entry__ as g; g.smoke()"
$S bench_$TAG 400 python3 bench.py
