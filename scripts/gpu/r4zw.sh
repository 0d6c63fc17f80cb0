#!/bin/bash
# round 4 final check on the last tree (after the lean transmit form's
# header windows and mask table, r4al): the door tests, the whole GPU suite,
# smoke, the default bench, transmit shapes and the lean form's HBM traffic at c2
set -u
S=scripts/gpu_step.sh
TAG=${1:-r4zw}
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONFAULTHANDLER=1
rm -f gpurun_out/.stop
$S pytest_door_$TAG 300 python -u -m pytest tests/test_gpu_door.py -x -q --timeout 120 --timeout-method thread
[ -f gpurun_out/.stop ] && exit 1
$S pytest_gpu_$TAG 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
[ -f gpurun_out/.stop ] && exit 1
$S smoke_$TAG 300 python3 scripts/smoke_run.py
[ -f gpurun_out/.stop ] && exit 1
$S bench_$TAG 400 python3 bench.py
[ -f gpurun_out/.stop ] && exit 1
for cfg in c2 c3 c4; do
  CONFIG=$cfg $S tx_${cfg}_$TAG 200 python3 scripts/bench_tx.py
  [ -f gpurun_out/.stop ] && exit 1
done
CONFIG=c2 REPS=2 $S pmcF_tx_c2_$TAG 180 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmcF_tx_c2_$TAG -o run --output-format csv -- python3 scripts/bench_tx.py
[ -f gpurun_out/.stop ] && exit 1
CONFIG=c2 REPS=2 $S pmcW_tx_c2_$TAG 180 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmcW_tx_c2_$TAG -o run --output-format csv -- python3 scripts/bench_tx.py
exit 0
