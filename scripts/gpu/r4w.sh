#!/bin/bash
# round 4: one transmit kernel (k_build_id gone), its geometry by mean frame
# size, timed from the tile index on -- transmit tests, c2/c3/c4 shapes,
# k_build HBM traffic at c2 and c3 (separate FETCH_SIZE / WRITE_SIZE passes),
# then the default bench (its tx leg) and the whole GPU suite
set -u
S=scripts/gpu_step.sh
TAG=${1:-r4w}
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONFAULTHANDLER=1
rm -f gpurun_out/.stop
$S pytest_tx_$TAG 400 python -u -m pytest tests/test_gpu_tx.py -x -q --timeout 120 --timeout-method thread
[ -f gpurun_out/.stop ] && exit 1
for cfg in c2 c3 c4; do
  CONFIG=$cfg $S tx_${cfg}_$TAG 200 python3 scripts/bench_tx.py
  [ -f gpurun_out/.stop ] && exit 1
done
for cfg in c2 c3; do
  CONFIG=$cfg REPS=2 $S pmcF_tx_${cfg}_$TAG 180 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmcF_tx_${cfg}_$TAG -o run --output-format csv -- python3 scripts/bench_tx.py
  [ -f gpurun_out/.stop ] && exit 1
  CONFIG=$cfg REPS=2 $S pmcW_tx_${cfg}_$TAG 180 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmcW_tx_${cfg}_$TAG -o run --output-format csv -- python3 scripts/bench_tx.py
  [ -f gpurun_out/.stop ] && exit 1
done
$S bench_$TAG 400 python3 bench.py
[ -f gpurun_out/.stop ] && exit 1
$S pytest_gpu_$TAG 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
exit 0
