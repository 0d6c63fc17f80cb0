#!/bin/bash
# r6u: c4 as one stream under a kernel trace -- is the step bound by the unmask
# (pieces back to back) or by the next batch's chain (gaps before a piece)?
set -u
S=scripts/gpu_step.sh
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
rm -f gpurun_out/.stop
$S c4one_kt_r6u 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6u_kt -o kt -- python3 bench.py --config c4 --segments 1 --steps 24 --warmup 4 --no-tx --feed-conns 0 --dropin-reads 0 --host-gib 0 --cpu-seconds 0
exit 0
