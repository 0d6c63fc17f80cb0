#!/bin/bash
# PMC counters of the frame sieve (c4 one stream): issue vs wait, LDS conflicts.
set -u
S=scripts/gpu_step.sh
export TMPDIR=/tmp
B="python bench.py --config c4 --segments 1 --cpu-seconds 0 --host-gib 0 --no-tx --steps 1 --warmup 0"
$S pmc_sq1 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU -d gpurun_out/pmc_sq1 -o run --output-format csv -- $B
$S pmc_sq2 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES -d gpurun_out/pmc_sq2 -o run --output-format csv -- $B
$S pmc_fetch 90 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- $B
