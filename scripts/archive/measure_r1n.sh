#!/bin/bash
# Host-inclusive chunk sizes; c2/c3 after the table-set sizing fix.
set -u
S=scripts/gpu_step.sh
TAG=${1:-r1n}
export TMPDIR=/tmp
$S bench_${TAG}_c2 300 python bench.py --config c2 --cpu-seconds 0 --host-gib 1 --no-tx
for m in 16 64 256; do
  $S bench_${TAG}_c3_chunk$m 300 python bench.py --cpu-seconds 0 --host-gib 4 --host-chunk-mib $m --no-tx --steps 4
done
