#!/bin/bash
# Round 2: is the ~20 us idle before a pipelined unmask a submission delay?
# c2 pipelined with HVWS_KICK 0/1/3 (hipStreamQuery on the unmask stream after
# queuing it / also while waiting for the check), interleaved, and a trace.
set -u
S=scripts/gpu_step.sh
TAG=${1:-r2k}
export TMPDIR=/tmp
rm -f gpurun_out/.stop
B="python3 bench.py --steps 200 --warmup 10 --cpu-seconds 0 --host-gib 0 --no-tx --config c2"
for rep in 1 2; do
  for k in 0 1 3; do
    HVWS_KICK=$k $S bench_${TAG}_c2_k${k}_$rep 200 $B
  done
done
HVWS_KICK=3 HVWS_STEP_EVENTS=0 $S trace_${TAG}_c2_k3 300 rocprofv3 --kernel-trace -d gpurun_out/trace_${TAG}_c2_k3 -o run --output-format csv -- python3 bench.py --config c2 --steps 20 --warmup 5 --cpu-seconds 0 --host-gib 0 --no-tx
