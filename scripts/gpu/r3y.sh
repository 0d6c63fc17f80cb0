#!/bin/bash
# round 3: rest of the closing pass (c4 one-stream step traffic, drop-in leg,
# N=2 rehearsal on one card), then the default bench under rocprofv3 with the
# resident worker off (exit crash under the profiler in r3v/r3x)
set -u
S=scripts/gpu_step.sh
TAG=${1:-r3y}
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
rm -f gpurun_out/.stop
# the worker now loads a request's first chunks beside the request itself
$S pytest_door_$TAG 300 python -u -m pytest tests/test_gpu_door.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "door or execute or message or decode or build_frame"
grep -q " passed" gpurun_out/pytest_door_$TAG.log && ! grep -q "failed" gpurun_out/pytest_door_$TAG.log || { echo "door tests not green"; exit 1; }
$S door_phases_$TAG 120 python3 scripts/probe/door_phases.py 2000
B4="python3 bench.py --config c4 --segments 1 --steps 30 --warmup 3 --cpu-seconds 0 --host-gib 0 --no-tx --feed-conns 0 --dropin-reads 0"
$S c4s1_$TAG 200 $B4
$S pmcF_c4s1_$TAG 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcF_c4s1_$TAG -o p -- $B4
$S pmcW_c4s1_$TAG 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmcW_c4s1_$TAG -o p -- $B4
$S dropin_$TAG 200 python3 scripts/bench_dropin.py 2000
HVWS_BENCH_WATCHDOG=60 HVWS_BENCH_DEVICE=0 $S rehearsal2_$TAG 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2
HVWS_DOOR=0 $S trace_door0_${TAG}_c3 300 rocprofv3 --kernel-trace --stats -d gpurun_out/trace_door0_${TAG}_c3 -o run --output-format csv -- python3 bench.py
