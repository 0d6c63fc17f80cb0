#!/bin/bash
# round 3 final tree: GPU suite and smoke (per-thread worker test opts in)
set -u
S=scripts/gpu_step.sh
TAG=${1:-r3ah}
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONFAULTHANDLER=1
rm -f gpurun_out/.stop
$S pytest_gpu_$TAG 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
[ -f gpurun_out/.stop ] && exit 1
$S smoke_$TAG 120 python3 -c "import __graft_entry__ as g; g.smoke()"
$S bench_$TAG 200 python3 bench.py
