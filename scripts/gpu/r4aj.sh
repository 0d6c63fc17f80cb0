#!/bin/bash
# round 4: SQ counters of the lean k_build form at the c2 shape (issue-bound
# or waiting?), two --pmc passes over scripts/bench_tx.py
set -u
S=scripts/gpu_step.sh
TAG=${1:-r4aj}
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONFAULTHANDLER=1
rm -f gpurun_out/.stop
CONFIG=c2 $S pmc1_tx_$TAG 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU -d gpurun_out/pmc1_tx_$TAG -o run --output-format csv -- python3 scripts/bench_tx.py
[ -f gpurun_out/.stop ] && exit 1
CONFIG=c2 $S pmc2_tx_$TAG 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_BUSY_CYCLES -d gpurun_out/pmc2_tx_$TAG -o run --output-format csv -- python3 scripts/bench_tx.py
exit 0
