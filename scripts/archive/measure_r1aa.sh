#!/bin/bash
# Walk register work: full GPU suite, c2/c3 benches, c2 trace.
set -u
S=scripts/gpu_step.sh
TAG=${1:-r1aa}
export TMPDIR=/tmp
$S pytest_gpu 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
$S bench_${TAG}_c2 300 python bench.py --config c2 --cpu-seconds 0 --host-gib 0 --no-tx
$S trace_${TAG}_c2 300 rocprofv3 --kernel-trace --stats -d gpurun_out/trace_${TAG}_c2 -o run --output-format csv -- python bench.py --config c2 --steps 5 --warmup 1 --cpu-seconds 0 --host-gib 0 --no-tx
$S bench_${TAG}_c4 300 python bench.py --config c4 --segments 1024 --cpu-seconds 0 --host-gib 0 --no-tx
