#!/bin/bash
# round 4: resident worker with the two-pass header walk and its request in
# device memory (large BAR) -- door tests, device phases and per-call latency
# against the speculative walk and the pinned request; transmit at the c2
# shape with 8 KiB (HVWS_BUILD=0) and 16 KiB (7) tiles and a kernel trace
# (k_tx_spans' cost); c2 with the walk's grid capped (HVWS_WALK_BLOCKS)
set -u
S=scripts/gpu_step.sh
TAG=${1:-r4d}
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONFAULTHANDLER=1
rm -f gpurun_out/.stop
$S pytest_door_$TAG 300 python -u -m pytest tests/test_gpu_door.py -x -q --timeout 120 --timeout-method thread
[ -f gpurun_out/.stop ] && exit 1
$S door_phases_$TAG 120 python3 scripts/probe/door_phases.py 2000
[ -f gpurun_out/.stop ] && exit 1
HVWS_DOOR_WALK=0 $S door_phases_walk0_$TAG 120 python3 scripts/probe/door_phases.py 2000
[ -f gpurun_out/.stop ] && exit 1
HVWS_DOOR_VRAM=0 $S door_phases_pinned_$TAG 120 python3 scripts/probe/door_phases.py 2000
[ -f gpurun_out/.stop ] && exit 1
$S dropin_$TAG 200 python3 scripts/bench_dropin.py 2000
[ -f gpurun_out/.stop ] && exit 1
for i in 1 2; do
  for b in 0 7; do
    CONFIG=c2 HVWS_BUILD=$b $S tx_c2_b${b}_${i}_$TAG 120 python3 scripts/bench_tx.py
    [ -f gpurun_out/.stop ] && exit 1
  done
done
CONFIG=c2 $S trace_tx_c2_$TAG 180 rocprofv3 --kernel-trace --stats -d gpurun_out/trace_tx_c2_$TAG -o run --output-format csv -- python3 scripts/bench_tx.py
[ -f gpurun_out/.stop ] && exit 1
C2="--config c2 --steps 200 --warmup 10 --no-tx --host-gib 0 --cpu-seconds 0 --feed-conns 0"
for wb in 0 256 512 0; do
  HVWS_WALK_BLOCKS=$wb $S c2_wb${wb}_$TAG 120 python3 bench.py $C2
  [ -f gpurun_out/.stop ] && exit 1
done
