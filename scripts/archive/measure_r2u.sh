#!/bin/bash
# Round 2 measurement pass: GPU suite, smoke, the default bench, the default
# bench under rocprofv3 --kernel-trace --stats, FETCH_SIZE / WRITE_SIZE in
# separate --pmc passes at c3.
set -u
S=scripts/gpu_step.sh
TAG=${1:-r2u}
export TMPDIR=/tmp
rm -f gpurun_out/.stop
$S pytest_gpu_$TAG 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
$S smoke_$TAG 120 python3 -c "import __graft_entry__ as g; g.smoke()"
$S bench_$TAG 400 python3 bench.py
$S trace_${TAG}_c3 500 rocprofv3 --kernel-trace --stats -d gpurun_out/trace_${TAG}_c3 -o run --output-format csv -- python3 bench.py
$S pmc_fetch_$TAG 400 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch_$TAG -o run --output-format csv -- python3 bench.py --steps 2 --warmup 0 --cpu-seconds 0 --host-gib 0
$S pmc_write_$TAG 400 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write_$TAG -o run --output-format csv -- python3 bench.py --steps 2 --warmup 0 --cpu-seconds 0 --host-gib 0
