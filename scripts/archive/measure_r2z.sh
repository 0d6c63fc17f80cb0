#!/bin/bash
# Round 2: GPU suite on the current tree (unmask-launch cleanup, transmit tests).
set -u
S=scripts/gpu_step.sh
TAG=${1:-r2z}
export TMPDIR=/tmp
rm -f gpurun_out/.stop
$S pytest_gpu_$TAG 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
$S smoke_$TAG 120 python3 -c "import __graft_entry__ as g; g.smoke()"
