#!/bin/bash
# Re-entry check of HEAD: GPU tests, smoke, default bench, c3 kernel trace.
set -u
S=scripts/gpu_step.sh
TAG=${1:-r1r}
export TMPDIR=/tmp
$S pytest_gpu 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
$S smoke_$TAG 200 python -c "import __graft_entry__ as g; g.smoke()"
$S bench_$TAG 400 python bench.py
$S trace_${TAG}_c3 300 rocprofv3 --kernel-trace --stats -d gpurun_out/trace_${TAG}_c3 -o run --output-format csv -- python bench.py --steps 5 --warmup 1 --cpu-seconds 0 --host-gib 0 --no-tx
