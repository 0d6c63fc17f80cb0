#!/bin/bash
# Round-1 second measurement pass: tests, bench (rx + tx), rocprof stats, PMC traffic.
set -u
S=scripts/gpu_step.sh
TAG=${1:-r1b}
export TMPDIR=/tmp
$S pytest_gpu 700 python -m pytest tests -m gpu -x -q
$S bench_$TAG 400 python bench.py
$S bench_${TAG}_c3_seg1 300 python bench.py --segments 1 --cpu-seconds 0 --host-gib 0 --steps 5
$S prof_${TAG} 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python bench.py --steps 5 --warmup 1 --cpu-seconds 0 --host-gib 0
$S pmc_fetch_${TAG} 400 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch_$TAG -o run --output-format csv -- python bench.py --steps 2 --warmup 0 --cpu-seconds 0 --host-gib 0
$S pmc_write_${TAG} 400 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write_$TAG -o run --output-format csv -- python bench.py --steps 2 --warmup 0 --cpu-seconds 0 --host-gib 0
$S feed_$TAG 300 python scripts/bench_feed.py
