#!/bin/bash
# r6ap: two ranks on one card with every leg of the default bench on except the
# transmit leg (two ranks' transmit buffers would not fit one card): the N > 1
# path of each leg (CPU baseline, host-inclusive, event loop, drop-in) as the
# driver's scaling run takes it, one rank per GPU there.
set -u
S=scripts/gpu_step.sh
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
rm -f gpurun_out/.stop
HVWS_BENCH_DEVICE=0 $S rehearsal_legs_r6ap 600 python3 bench.py --gpus 2 --no-tx
exit 0
