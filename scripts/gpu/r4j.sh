#!/bin/bash
# round 4: the resident worker on by default and bench.py's drop-in leg on by
# default -- door tests, the whole GPU suite, smoke, the default bench twice,
# the default bench under a kernel trace; then k_build's SQ counters at the
# c2 shape (two passes)
set -u
S=scripts/gpu_step.sh
TAG=${1:-r4j}
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONFAULTHANDLER=1
rm -f gpurun_out/.stop
$S pytest_door_$TAG 300 python -u -m pytest tests/test_gpu_door.py -x -q --timeout 120 --timeout-method thread
[ -f gpurun_out/.stop ] && exit 1
$S pytest_gpu_$TAG 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
[ -f gpurun_out/.stop ] && exit 1
$S smoke_$TAG 300 python3 scripts/smoke_run.py
[ -f gpurun_out/.stop ] && exit 1
for i in 1 2; do
  $S bench_${i}_$TAG 400 python3 bench.py
  [ -f gpurun_out/.stop ] && exit 1
done
$S trace_c3_$TAG 400 rocprofv3 --kernel-trace --stats -d gpurun_out/trace_c3_$TAG -o run --output-format csv -- python3 bench.py
[ -f gpurun_out/.stop ] && exit 1
CONFIG=c2 $S pmc1_tx_$TAG 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU -d gpurun_out/pmc1_tx_$TAG -o run --output-format csv -- python3 scripts/bench_tx.py
[ -f gpurun_out/.stop ] && exit 1
CONFIG=c2 $S pmc2_tx_$TAG 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_BUSY_CYCLES -d gpurun_out/pmc2_tx_$TAG -o run --output-format csv -- python3 scripts/bench_tx.py
exit 0
