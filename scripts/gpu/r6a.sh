#!/bin/bash
# r6a: the exit crash under rocprofv3 with a worker stream alive:
# the same one-read process unprofiled (must exit 0), then traced, with its maps.
set -u
S=scripts/gpu_step.sh
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
rm -f gpurun_out/.stop
$S exit_plain_r6a 60 python3 scripts/probe/exit_probe.py plain_r6a
[ -f gpurun_out/.stop ] && exit 1
$S exit_kt_r6a 90 rocprofv3 --kernel-trace --stats -d gpurun_out/r6a_kt -o kt -- python3 scripts/probe/exit_probe.py kt_r6a
exit 0
