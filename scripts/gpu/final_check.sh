#!/bin/bash
# The driver's round-end commands on the final tree: the GPU suite, smoke, the default bench
set -u
S=scripts/gpu_step.sh
TAG=${1:-final}
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONFAULTHANDLER=1
rm -f gpurun_out/.stop
$S pytest_gpu_$TAG 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
[ -f gpurun_out/.stop ] && exit 1
$S smoke_$TAG 300 python3 scripts/smoke_run.py
[ -f gpurun_out/.stop ] && exit 1
$S bench_$TAG 400 python3 bench.py
exit 0
