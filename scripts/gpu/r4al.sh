#!/bin/bash
# round 4: lean k_build with each frame's header bytes pre-placed in its two
# output chunks and payload bytes kept by a byte-mask table (no per-chunk
# shifts into place; 161 -> 90 VALU per chunk in the assembly) -- transmit
# tests (lean forced too), c2 three times, c3 / c4 once, SQ VALU counters
set -u
S=scripts/gpu_step.sh
TAG=${1:-r4al}
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONFAULTHANDLER=1
rm -f gpurun_out/.stop
$S pytest_tx_$TAG 400 python -u -m pytest tests/test_gpu_tx.py -x -q --timeout 120 --timeout-method thread
[ -f gpurun_out/.stop ] && exit 1
HVWS_BUILD=5 $S pytest_tx_b5_$TAG 400 python -u -m pytest tests/test_gpu_tx.py -x -q --timeout 120 --timeout-method thread -k "not every_geometry and not by_frame_size"
[ -f gpurun_out/.stop ] && exit 1
for rep in 1 2 3; do
  CONFIG=c2 $S tx_c2_${rep}_$TAG 200 python3 scripts/bench_tx.py
  [ -f gpurun_out/.stop ] && exit 1
done
for cfg in c3 c4; do
  CONFIG=$cfg $S tx_${cfg}_$TAG 200 python3 scripts/bench_tx.py
  [ -f gpurun_out/.stop ] && exit 1
done
CONFIG=c2 $S pmc1_tx_$TAG 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU -d gpurun_out/pmc1_tx_$TAG -o run --output-format csv -- python3 scripts/bench_tx.py
exit 0
