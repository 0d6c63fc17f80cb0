#!/bin/bash
# round 4, resident worker v2 (request block and bytes in fine-grained device
# memory written through the BAR) against v1 (pinned host, HVWS_DOOR_VRAM=0):
# door tests both ways, ASan exit path, device phases and per-call latency
# both ways, the serial door walk against the speculative one (HVWS_DOOR_WALK=0),
# then the whole GPU suite with the worker on (HVWS_DOOR=1)
set -u
S=scripts/gpu_step.sh
TAG=${1:-r4c}
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONFAULTHANDLER=1
rm -f gpurun_out/.stop
$S pytest_door_v2_$TAG 300 python -u -m pytest tests/test_gpu_door.py -x -q --timeout 120 --timeout-method thread
[ -f gpurun_out/.stop ] && exit 1
HVWS_DOOR_VRAM=0 $S pytest_door_v1_$TAG 300 python -u -m pytest tests/test_gpu_door.py -x -q --timeout 120 --timeout-method thread
[ -f gpurun_out/.stop ] && exit 1
ASAN_OPTIONS=detect_leaks=0 $S asan_door_$TAG 180 build/asan/asan_driver door
[ -f gpurun_out/.stop ] && exit 1
for v in 1 0; do
  HVWS_DOOR_VRAM=$v $S door_phases_v${v}_$TAG 120 python3 scripts/probe/door_phases.py 2000
  [ -f gpurun_out/.stop ] && exit 1
  HVWS_DOOR_VRAM=$v $S dropin_v${v}_$TAG 200 python3 scripts/bench_dropin.py 2000
  [ -f gpurun_out/.stop ] && exit 1
done
HVWS_DOOR_WALK=0 $S door_phases_walk0_$TAG 120 python3 scripts/probe/door_phases.py 2000
[ -f gpurun_out/.stop ] && exit 1
HVWS_DOOR_WALK=0 $S dropin_walk0_$TAG 200 python3 scripts/bench_dropin.py 2000
[ -f gpurun_out/.stop ] && exit 1
HVWS_DOOR=1 $S pytest_gpu_door_on_$TAG 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
