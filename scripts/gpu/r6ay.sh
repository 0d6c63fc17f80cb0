#!/bin/bash
# r6ay: SQ instruction counts of the final worker (tree) against the r6z3 tree's
# (build/ab/libhvws_r6z3.so), 4000 reads of door_phases.py each
set -u
S=scripts/gpu_step.sh
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
rm -f gpurun_out/.stop
A="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY"
$S sqA_new_r6ay 150 timeout -s KILL 120 rocprofv3 --pmc $A -d gpurun_out/r6ay_sqA_new -o sq -- python3 scripts/probe/door_phases.py 4000
[ -f gpurun_out/.stop ] && exit 1
HVWS_LIB=build/ab/libhvws_r6z3.so $S sqA_old_r6ay 150 timeout -s KILL 120 rocprofv3 --pmc $A -d gpurun_out/r6ay_sqA_old -o sq -- python3 scripts/probe/door_phases.py 4000
exit 0
