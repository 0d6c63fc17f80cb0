#!/bin/bash
# round 3: the other configs' bench lines on the final tree (c2 with its
# transmit leg, c4 with 1024 connections), then the full GPU suite
set -u
S=scripts/gpu_step.sh
TAG=${1:-r3z}
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
rm -f gpurun_out/.stop
$S c2_$TAG 200 python3 bench.py --config c2 --steps 100 --warmup 5 --cpu-seconds 0 --host-gib 0 --feed-conns 0 --dropin-reads 0
$S c4_$TAG 200 python3 bench.py --config c4 --segments 1024 --steps 30 --warmup 3 --cpu-seconds 0 --host-gib 0 --feed-conns 0 --dropin-reads 0
$S c4s1_$TAG 200 python3 bench.py --config c4 --segments 1 --steps 30 --warmup 3 --cpu-seconds 0 --host-gib 0 --feed-conns 0 --dropin-reads 0
$S pytest_gpu_$TAG 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
$S smoke_$TAG 120 python3 -c "import __graft_entry__ as g; g.smoke()"
$S bench_$TAG 300 python3 bench.py
