#!/bin/bash
# round 4: c4 as one stream with the one-wave unmask capped at 12 workgroups
# per CU (the chain beside it is now the longer one): regions of 160 / 192 /
# 224 / 256 frames ($HVWS_SIEVE_HOPS; shorter link walks, more window bytes)
set -u
S=scripts/gpu_step.sh
TAG=${1:-r4z}
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONFAULTHANDLER=1
rm -f gpurun_out/.stop
L="--steps 20 --warmup 3 --cpu-seconds 0 --host-gib 0 --no-tx --feed-conns 0 --dropin-reads 0"
for h in 256 192 160 224; do
  HVWS_UNMASK=12 HVWS_UNMASK_LDS=3072 HVWS_SIEVE_HOPS=$h $S c4s1_u12_h${h}_$TAG 200 python3 bench.py --config c4 --segments 1 $L
  [ -f gpurun_out/.stop ] && exit 1
  HVWS_SIEVE_HOPS=$h $S c4s1_def_h${h}_$TAG 200 python3 bench.py --config c4 --segments 1 $L
  [ -f gpurun_out/.stop ] && exit 1
done
exit 0
