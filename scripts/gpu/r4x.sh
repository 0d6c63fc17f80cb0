#!/bin/bash
# round 4: the unmask with one-wave workgroups (12: 64 x 4, 13: 64 x 8,
# 14: 64 x 16, linear) against the 512 x 2 default below 16 GiB (11), in
# pipelined steps beside the next batch's scan: c2, c4 (1024 connections),
# c4 as one stream; light bench runs (device legs only)
set -u
S=scripts/gpu_step.sh
TAG=${1:-r4x}
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONFAULTHANDLER=1
rm -f gpurun_out/.stop
L="--steps 20 --warmup 3 --cpu-seconds 0 --host-gib 0 --no-tx --feed-conns 0 --dropin-reads 0"
for i in 1 2; do
  for v in 11 12 13 14; do
    HVWS_UNMASK=$v $S c2_u${v}_${i}_$TAG 200 python3 bench.py --config c2 $L
    [ -f gpurun_out/.stop ] && exit 1
  done
done
for v in 11 12 13; do
  HVWS_UNMASK=$v $S c4_u${v}_$TAG 200 python3 bench.py --config c4 --segments 1024 $L
  [ -f gpurun_out/.stop ] && exit 1
  HVWS_UNMASK=$v $S c4s1_u${v}_$TAG 200 python3 bench.py --config c4 --segments 1 $L
  [ -f gpurun_out/.stop ] && exit 1
done
exit 0
