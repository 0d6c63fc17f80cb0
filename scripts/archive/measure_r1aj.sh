#!/bin/bash
set -u
S=scripts/gpu_step.sh
export TMPDIR=/tmp
B="python bench.py --config c2 --cpu-seconds 0 --host-gib 0 --no-tx --steps 2 --warmup 0 --serial"
$S aj_pmc1 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU -d gpurun_out/aj_pmc1 -o run --output-format csv -- $B
$S aj_pmc2 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES TA_BUSY_avr TA_TA_BUSY_sum -d gpurun_out/aj_pmc2 -o run --output-format csv -- $B
$S aj_trace 200 rocprofv3 --kernel-trace --stats -d gpurun_out/aj_trace -o run --output-format csv -- $B
