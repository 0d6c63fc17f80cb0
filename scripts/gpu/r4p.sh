#!/bin/bash
# round 4: k_build_uni with reciprocal divisions; worker streams pooled per
# device; bounded worker-stream drains.  Door tests (a stuck thread dumps
# native stacks and mailboxes), ASan of the worker's exit paths, transmit
# shapes, then a whole pass: GPU suite, smoke, default bench, the 2-rank
# rehearsal on one card, the default bench under a kernel trace, the
# worker's phases and per-call latency
set -u
S=scripts/gpu_step.sh
TAG=${1:-r4p}
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONFAULTHANDLER=1
rm -f gpurun_out/.stop
$S pytest_door_$TAG 300 python -u -m pytest tests/test_gpu_door.py -x -v --timeout 120 --timeout-method thread
[ -f gpurun_out/.stop ] && exit 1
ASAN_OPTIONS=detect_leaks=0 $S asan_door_$TAG 180 build/asan/asan_driver door
[ -f gpurun_out/.stop ] && exit 1
$S pytest_tx_$TAG 400 python -u -m pytest tests/test_gpu_tx.py -x -q --timeout 120 --timeout-method thread
[ -f gpurun_out/.stop ] && exit 1
for i in 1 2; do
  CONFIG=c2 $S tx_c2_${i}_$TAG 120 python3 scripts/bench_tx.py
  [ -f gpurun_out/.stop ] && exit 1
done
CONFIG=c3 $S tx_c3_$TAG 200 python3 scripts/bench_tx.py
[ -f gpurun_out/.stop ] && exit 1
$S pytest_gpu_$TAG 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
[ -f gpurun_out/.stop ] && exit 1
$S smoke_$TAG 300 python3 scripts/smoke_run.py
[ -f gpurun_out/.stop ] && exit 1
$S bench_$TAG 400 python3 bench.py
[ -f gpurun_out/.stop ] && exit 1
HVWS_BENCH_DEVICE=0 $S rehearsal2_$TAG 600 python3 bench.py --gpus 2
[ -f gpurun_out/.stop ] && exit 1
$S trace_c3_$TAG 400 rocprofv3 --kernel-trace --stats -d gpurun_out/trace_c3_$TAG -o run --output-format csv -- python3 bench.py
[ -f gpurun_out/.stop ] && exit 1
$S door_phases_$TAG 120 python3 scripts/probe/door_phases.py 2000
[ -f gpurun_out/.stop ] && exit 1
$S dropin_$TAG 200 python3 scripts/bench_dropin.py 2000
exit 0
