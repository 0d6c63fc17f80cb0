#!/bin/bash
# round 4: one-wave unmask workgroups capped per CU by dynamic LDS (20 KiB a
# workgroup: 8 per CU; 13 KiB: 12) against the default, pipelined steps at
# c2 and c4 as one stream (device legs only)
set -u
S=scripts/gpu_step.sh
TAG=${1:-r4y}
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONFAULTHANDLER=1
rm -f gpurun_out/.stop
L="--steps 20 --warmup 3 --cpu-seconds 0 --host-gib 0 --no-tx --feed-conns 0 --dropin-reads 0"
for cfg in "c2 4096" "c4 1"; do
  set -- $cfg
  $S ${1}s${2}_def_$TAG 200 python3 bench.py --config $1 --segments $2 $L
  [ -f gpurun_out/.stop ] && exit 1
  for v in 12 14; do
    for lds in 10240 3072; do
      HVWS_UNMASK=$v HVWS_UNMASK_LDS=$lds $S ${1}s${2}_u${v}_l${lds}_$TAG 200 python3 bench.py --config $1 --segments $2 $L
      [ -f gpurun_out/.stop ] && exit 1
    done
  done
  $S ${1}s${2}_def2_$TAG 200 python3 bench.py --config $1 --segments $2 $L
  [ -f gpurun_out/.stop ] && exit 1
done
exit 0
