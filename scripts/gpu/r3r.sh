#!/bin/bash
# round 3 (session 2): pass on the restored tree -- GPU suite, smoke, default
# bench, default bench under rocprofv3 --kernel-trace --stats
set -u
S=scripts/gpu_step.sh
TAG=${1:-r3r}
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
rm -f gpurun_out/.stop
$S pytest_gpu_$TAG 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
$S smoke_$TAG 120 python3 -c "import __graft_entry__ as g; g.smoke()"
$S bench_$TAG 400 python3 bench.py
$S trace_${TAG}_c3 500 rocprofv3 --kernel-trace --stats -d gpurun_out/trace_${TAG}_c3 -o run --output-format csv -- python3 bench.py
