#!/bin/bash
# r6an: the final worker (8 waves, HSA queue) through 100 fresh processes that
# make one read and release their context 0-12 ms later (door_first), and the
# traced exit probes under rocprofv3.
set -u
S=scripts/gpu_step.sh
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
rm -f gpurun_out/.stop
$S door_first_r6an 500 bash scripts/probe/door_first.sh run 100
[ -f gpurun_out/.stop ] && exit 1
EXIT_PROBE_MAPS=0 $S exit_kt_r6an 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r6an_exit -o kt -- python3 scripts/probe/exit_probe.py test
exit 0
