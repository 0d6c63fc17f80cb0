#!/bin/bash
# Round 2: XCD-chunked tile orders (variants 12-15).  The all-geometry parity
# test, then bench --sweep-unmask (every geometry interleaved in one process,
# unmask and in-place stream rates) at c2, c4 (1024 segments) and c3, and
# pipelined c2/c4 runs of the chunked variants against the current choice.
set -u
S=scripts/gpu_step.sh
TAG=${1:-r2s}
export TMPDIR=/tmp
rm -f gpurun_out/.stop
$S geomtest_$TAG 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "unmask_geometries or speculative_table"
B="python3 bench.py --cpu-seconds 0 --host-gib 0 --no-tx"
$S sweep_${TAG}_c2 300 $B --config c2 --steps 2 --warmup 1 --sweep-unmask
$S sweep_${TAG}_c4 300 $B --config c4 --segments 1024 --steps 2 --warmup 1 --sweep-unmask
$S sweep_${TAG}_c3 600 $B --steps 2 --warmup 1 --sweep-unmask
for v in 11 13 15; do
  HVWS_UNMASK=$v $S bench_${TAG}_c2_u$v 200 $B --steps 200 --warmup 10 --config c2
done
for v in 11 13 15; do
  HVWS_UNMASK=$v $S bench_${TAG}_c4_u$v 200 $B --steps 100 --warmup 10 --config c4 --segments 1024
done
