#!/bin/bash
# round 3 closing pass on the final tree: GPU suite, smoke, default bench,
# the default bench under rocprofv3 --kernel-trace --stats, c4 one stream, the
# drop-in leg; stops at the first crash
set -u
S=scripts/gpu_step.sh
TAG=${1:-r3ac}
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONFAULTHANDLER=1
rm -f gpurun_out/.stop
$S pytest_gpu_$TAG 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
[ -f gpurun_out/.stop ] && exit 1
$S smoke_$TAG 120 python3 -c "import __graft_entry__ as g; g.smoke()"
$S bench_$TAG 300 python3 bench.py
[ -f gpurun_out/.stop ] && exit 1
$S trace_${TAG}_c3 300 rocprofv3 --kernel-trace --stats -d gpurun_out/trace_${TAG}_c3 -o run --output-format csv -- python3 bench.py
[ -f gpurun_out/.stop ] && exit 1
$S c4s1_$TAG 200 python3 bench.py --config c4 --segments 1 --steps 30 --warmup 3 --cpu-seconds 0 --host-gib 0 --feed-conns 0 --dropin-reads 0
$S c2_$TAG 200 python3 bench.py --config c2 --steps 100 --warmup 5 --cpu-seconds 0 --host-gib 0 --feed-conns 0 --dropin-reads 0
