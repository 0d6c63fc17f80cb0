#!/bin/bash
# round 4, first pass: the 2-rank rehearsal through bench.py's own launcher
# (both ranks on card 0), then the default N=1 bench
set -u
S=scripts/gpu_step.sh
TAG=${1:-r4a}
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONFAULTHANDLER=1
rm -f gpurun_out/.stop
HVWS_BENCH_DEVICE=0 $S rehearsal2_$TAG 500 python3 bench.py --gpus 2
[ -f gpurun_out/.stop ] && exit 1
$S bench_$TAG 300 python3 bench.py
