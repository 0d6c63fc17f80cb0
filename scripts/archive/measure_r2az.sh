#!/bin/bash
# Round 2 closing pass (feeder, in-place pinned reads): GPU suite, smoke, the
# default bench, the default bench under rocprofv3 --kernel-trace --stats
# (no PMC pass: k_unmask is unchanged since profiles/traffic.json).
set -u
S=scripts/gpu_step.sh
TAG=${1:-r2az}
export TMPDIR=/tmp
rm -f gpurun_out/.stop
$S pytest_gpu_$TAG 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
$S smoke_$TAG 120 python3 -c "import __graft_entry__ as g; g.smoke()"
$S bench_$TAG 400 python3 bench.py
$S trace_${TAG}_c3 500 rocprofv3 --kernel-trace --stats -d gpurun_out/trace_${TAG}_c3 -o run --output-format csv -- python3 bench.py
