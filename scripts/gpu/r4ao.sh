#!/bin/bash
# round 4: kernel trace of the transmit bench at the c2 shape (lean form) on
# the final tree, for the rocprof summary of k_build<64x4,lean>
set -u
S=scripts/gpu_step.sh
TAG=${1:-r4ao}
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONFAULTHANDLER=1
rm -f gpurun_out/.stop
CONFIG=c2 $S trace_tx_c2_$TAG 200 rocprofv3 --kernel-trace --stats -d gpurun_out/trace_tx_c2_$TAG -o run --output-format csv -- python3 scripts/bench_tx.py
exit 0
