#!/bin/bash
# round 4 closing pass, second (after the lean transmit form stopped spilling
# and the sieve's prefetch fix): door tests, ASan of the worker's exit paths,
# the whole GPU suite, smoke, the default bench twice, the 2-rank rehearsal on
# one card, the default bench under a kernel trace (released worker streams
# destroyed), the worker's phases and per-call latency,
# transmit shapes and the lean form's HBM traffic, the c2 / c4 / c4 one-stream legs
set -u
S=scripts/gpu_step.sh
TAG=${1:-r4zy}
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONFAULTHANDLER=1
rm -f gpurun_out/.stop
$S pytest_door_$TAG 300 python -u -m pytest tests/test_gpu_door.py -x -v --timeout 120 --timeout-method thread
[ -f gpurun_out/.stop ] && exit 1
ASAN_OPTIONS=detect_leaks=0 $S asan_door_$TAG 180 build/asan/asan_driver door
[ -f gpurun_out/.stop ] && exit 1
$S pytest_gpu_$TAG 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
[ -f gpurun_out/.stop ] && exit 1
$S smoke_$TAG 300 python3 scripts/smoke_run.py
[ -f gpurun_out/.stop ] && exit 1
for i in 1 2; do
  $S bench_${i}_$TAG 400 python3 bench.py
  [ -f gpurun_out/.stop ] && exit 1
done
HVWS_BENCH_DEVICE=0 $S rehearsal2_$TAG 600 python3 bench.py --gpus 2
[ -f gpurun_out/.stop ] && exit 1
HVWS_DOOR_POOL=0 $S trace_c3_$TAG 400 rocprofv3 --kernel-trace --stats -d gpurun_out/trace_c3_$TAG -o run --output-format csv -- python3 bench.py
[ -f gpurun_out/.stop ] && exit 1
$S door_phases_$TAG 120 python3 scripts/probe/door_phases.py 2000
[ -f gpurun_out/.stop ] && exit 1
$S dropin_$TAG 200 python3 scripts/bench_dropin.py 2000
[ -f gpurun_out/.stop ] && exit 1
for cfg in c2 c3 c4; do
  CONFIG=$cfg $S tx_${cfg}_$TAG 200 python3 scripts/bench_tx.py
  [ -f gpurun_out/.stop ] && exit 1
done
CONFIG=c2 REPS=2 $S pmcF_tx_c2_$TAG 180 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmcF_tx_c2_$TAG -o run --output-format csv -- python3 scripts/bench_tx.py
[ -f gpurun_out/.stop ] && exit 1
CONFIG=c2 REPS=2 $S pmcW_tx_c2_$TAG 180 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmcW_tx_c2_$TAG -o run --output-format csv -- python3 scripts/bench_tx.py
[ -f gpurun_out/.stop ] && exit 1
L="--steps 20 --warmup 3 --cpu-seconds 0 --host-gib 0 --no-tx --feed-conns 0 --dropin-reads 0"
$S c2_$TAG 200 python3 bench.py --config c2 $L
[ -f gpurun_out/.stop ] && exit 1
$S c4_$TAG 200 python3 bench.py --config c4 --segments 1024 $L
[ -f gpurun_out/.stop ] && exit 1
$S c4s1_$TAG 200 python3 bench.py --config c4 --segments 1 $L
exit 0
