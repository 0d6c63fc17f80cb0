#!/bin/bash
# round 3: the worker-hang probe (scripts/probe/door_stress.py) under a short
# time limit; nothing runs after it
set -u
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONFAULTHANDLER=1
mkdir -p gpurun_out
HVWS_DOOR=1 timeout -k 10 150 python3 -u scripts/probe/door_stress.py 30 > gpurun_out/door_stress_r3ai.log 2>&1
echo "rc=$?"
tail -8 gpurun_out/door_stress_r3ai.log
