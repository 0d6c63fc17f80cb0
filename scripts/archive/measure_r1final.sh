#!/bin/bash
# End-of-round pass: GPU suite, smoke, default bench (c3) untraced and under a
# kernel trace (the traced process's JSON line and its trace agree by
# construction), c2 / c4 (1024 connections) / c4 one stream, c3 one stream.
set -u
S=scripts/gpu_step.sh
TAG=${1:-r1f}
export TMPDIR=/tmp
$S pytest_gpu 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
$S smoke_$TAG 200 python -c "import __graft_entry__ as g; g.smoke()"
$S bench_$TAG 400 python bench.py
$S trace_${TAG}_c3 500 rocprofv3 --kernel-trace --stats -d gpurun_out/trace_${TAG}_c3 -o run --output-format csv -- python bench.py
$S bench_${TAG}_c2 300 python bench.py --config c2 --cpu-seconds 2 --host-gib 1
$S bench_${TAG}_c4 300 python bench.py --config c4 --segments 1024 --cpu-seconds 2 --host-gib 1
$S bench_${TAG}_c4_seg1 300 python bench.py --config c4 --segments 1 --cpu-seconds 0 --host-gib 0 --no-tx
$S bench_${TAG}_c3_seg1 300 python bench.py --segments 1 --cpu-seconds 0 --host-gib 0 --no-tx --steps 5
