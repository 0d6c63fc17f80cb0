#!/bin/bash
# round 4, first pass: hipStreamQuery probe (does "idle" ever precede the
# kernel's own last store?), the GPU suite after the FUSED / k_pscan removal
# and the worker's epoch protocol, the 2-rank rehearsal through bench.py's own
# launcher (both ranks on card 0), then the default N=1 bench
set -u
S=scripts/gpu_step.sh
TAG=${1:-r4a}
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONFAULTHANDLER=1
rm -f gpurun_out/.stop
$S query_probe_$TAG 120 build/query_probe 300
[ -f gpurun_out/.stop ] && exit 1
$S vram_probe_$TAG 120 build/vram_probe
[ -f gpurun_out/.stop ] && exit 1
$S pytest_door_$TAG 300 python -u -m pytest tests/test_gpu_door.py -x -v --timeout 120 --timeout-method thread
[ -f gpurun_out/.stop ] && exit 1
ASAN_OPTIONS=detect_leaks=0 $S asan_door_$TAG 180 build/asan/asan_driver door
[ -f gpurun_out/.stop ] && exit 1
$S pytest_gpu_$TAG 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
[ -f gpurun_out/.stop ] && exit 1
HVWS_BENCH_DEVICE=0 $S rehearsal2_$TAG 500 python3 bench.py --gpus 2
[ -f gpurun_out/.stop ] && exit 1
$S bench_$TAG 300 python3 bench.py
