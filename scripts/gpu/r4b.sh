#!/bin/bash
# round 4, c2 and transmit pass: pipelined c2 with the unmask queued behind a
# cross-stream event (HVWS_HOST_ORDER=0, round 3) vs after the host saw the
# scan finish (default), interleaved; c2 step traffic (two --pmc passes) and a
# kernel trace; transmit at the c2 shape, boundary tiles records-first
# (HVWS_BUILD_SPANS=0) vs span-staged (default), interleaved; c4 as one
# stream without (HVWS_SIEVE_STOP=0) and with the window early stop
set -u
S=scripts/gpu_step.sh
TAG=${1:-r4b}
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONFAULTHANDLER=1
rm -f gpurun_out/.stop
C2="--config c2 --steps 200 --warmup 10 --no-tx --host-gib 0 --cpu-seconds 0 --feed-conns 0"
for i in 1 2; do
  for ho in 0 1; do
    HVWS_HOST_ORDER=$ho $S c2_ho${ho}_${i}_$TAG 120 python3 bench.py $C2
    [ -f gpurun_out/.stop ] && exit 1
  done
done
for i in 1 2; do
  for sp in 0 1; do
    CONFIG=c2 HVWS_BUILD_SPANS=$sp $S tx_c2_sp${sp}_${i}_$TAG 120 python3 scripts/bench_tx.py
    [ -f gpurun_out/.stop ] && exit 1
  done
done
C4="--config c4 --segments 1 --steps 100 --warmup 10 --no-tx --host-gib 0 --cpu-seconds 0 --feed-conns 0"
for i in 1 2; do
  for ss in 0 1; do
    HVWS_SIEVE_STOP=$ss $S c4s1_stop${ss}_${i}_$TAG 150 python3 bench.py $C4
    [ -f gpurun_out/.stop ] && exit 1
  done
done
P2="--config c2 --steps 30 --warmup 5 --no-tx --host-gib 0 --cpu-seconds 0 --feed-conns 0"
$S trace_c2_$TAG 180 rocprofv3 --kernel-trace --stats -d gpurun_out/trace_c2_$TAG -o run --output-format csv -- python3 bench.py $P2
[ -f gpurun_out/.stop ] && exit 1
$S pmcF_c2_$TAG 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmcF_c2_$TAG -o run --output-format csv -- python3 bench.py $P2
[ -f gpurun_out/.stop ] && exit 1
$S pmcW_c2_$TAG 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmcW_c2_$TAG -o run --output-format csv -- python3 bench.py $P2
