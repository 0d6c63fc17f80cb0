#!/bin/bash
# r6l: where the worker's read spends its cycles -- SQ counters over the
# worker's dispatch (4000 reads of door_phases.py; per read = total / 4000),
# the restructured worker (tree) against HEAD's (build/ab/libhvws_head.so).
set -u
S=scripts/gpu_step.sh
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
rm -f gpurun_out/.stop
A="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY"
B="SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS"
$S sqA_new_r6l 150 timeout -s KILL 120 rocprofv3 --pmc $A -d gpurun_out/r6l_sqA_new -o sq -- python3 scripts/probe/door_phases.py 4000
[ -f gpurun_out/.stop ] && exit 1
HVWS_LIB=build/ab/libhvws_head.so $S sqA_old_r6l 150 timeout -s KILL 120 rocprofv3 --pmc $A -d gpurun_out/r6l_sqA_old -o sq -- python3 scripts/probe/door_phases.py 4000
[ -f gpurun_out/.stop ] && exit 1
$S sqB_new_r6l 150 timeout -s KILL 120 rocprofv3 --pmc $B -d gpurun_out/r6l_sqB_new -o sq -- python3 scripts/probe/door_phases.py 4000
[ -f gpurun_out/.stop ] && exit 1
HVWS_LIB=build/ab/libhvws_head.so $S sqB_old_r6l 150 timeout -s KILL 120 rocprofv3 --pmc $B -d gpurun_out/r6l_sqB_old -o sq -- python3 scripts/probe/door_phases.py 4000
exit 0
