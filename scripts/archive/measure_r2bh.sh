#!/bin/bash
# Round 2 final pass: GPU suite, smoke, default bench (with the event-loop
# leg), the event-loop bench, then the default bench under rocprofv3
# --kernel-trace --stats.
set -u
S=scripts/gpu_step.sh
TAG=${1:-r2bh}
export TMPDIR=/tmp
rm -f gpurun_out/.stop
$S pytest_gpu_$TAG 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
$S smoke_$TAG 120 python3 -c "import __graft_entry__ as g; g.smoke()"
$S bench_$TAG 400 python3 bench.py
MODES=gpu_many,gpu_pipe,gpu_many_ring,gpu_pipe_ring,cpu_ref CONNS=1,16,64,256,1024,4096 $S benchfeed_$TAG 300 python3 -u scripts/bench_feed.py
$S trace_${TAG}_c3 500 rocprofv3 --kernel-trace --stats -d gpurun_out/trace_${TAG}_c3 -o run --output-format csv -- python3 bench.py
