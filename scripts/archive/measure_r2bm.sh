#!/bin/bash
# Round 2, final tree: the other BASELINE configs through bench.py (c2 1 KiB
# frames, c4 mixed as 1024 connections and as one stream), default c3 beside.
set -u
S=scripts/gpu_step.sh
TAG=${1:-r2bm}
export TMPDIR=/tmp
rm -f gpurun_out/.stop
B="python3 bench.py --cpu-seconds 0 --host-gib 0 --no-tx --feed-conns 0"
$S bench_${TAG}_c3 300 $B --steps 20 --warmup 5
$S bench_${TAG}_c2 200 $B --steps 200 --warmup 10 --config c2
$S bench_${TAG}_c4 200 $B --steps 100 --warmup 10 --config c4 --segments 1024
$S bench_${TAG}_c4one 200 $B --steps 50 --warmup 5 --config c4 --segments 1
