#!/bin/bash
# Round 2: after the unmask-launch cleanup: GPU suite, smoke, default bench, c2/c4.
set -u
S=scripts/gpu_step.sh
TAG=${1:-r2w}
export TMPDIR=/tmp
rm -f gpurun_out/.stop
$S pytest_gpu_$TAG 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
$S smoke_$TAG 120 python3 -c "import __graft_entry__ as g; g.smoke()"
$S bench_$TAG 400 python3 bench.py --steps 20 --warmup 5
B="python3 bench.py --cpu-seconds 0 --host-gib 0 --no-tx"
$S bench_${TAG}_c2 200 $B --steps 200 --warmup 10 --config c2
$S bench_${TAG}_c4 200 $B --steps 100 --warmup 10 --config c4 --segments 1024
