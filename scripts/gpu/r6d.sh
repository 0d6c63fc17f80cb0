#!/bin/bash
# r6d: bisect the exit crash under rocprofv3 -- no worker at all; the worker
# streams synchronised at exit; destroyed at exit (each traced; a crash ends the call).
set -u
S=scripts/gpu_step.sh
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
rm -f gpurun_out/.stop
P="python3 scripts/probe/exit_probe.py"
HVWS_DOOR=0 $S exit_nodoor_r6d 60 rocprofv3 --kernel-trace --stats -d gpurun_out/r6d_kt_nodoor -o kt -- $P nodoor_r6d
[ -f gpurun_out/.stop ] && exit 1
HVWS_EXPERIMENT=exit_door=2 $S exit_destroy_plain_r6d 60 $P destroyp_r6d
[ -f gpurun_out/.stop ] && exit 1
HVWS_EXPERIMENT=exit_door=2 $S exit_destroy_kt_r6d 60 rocprofv3 --kernel-trace --stats -d gpurun_out/r6d_kt_destroy -o kt -- $P destroy_r6d
[ -f gpurun_out/.stop ] && exit 1
HVWS_EXPERIMENT=exit_door=1 $S exit_sync_kt_r6d 60 rocprofv3 --kernel-trace --stats -d gpurun_out/r6d_kt_sync -o kt -- $P sync_r6d
exit 0
