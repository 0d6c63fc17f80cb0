#!/bin/bash
# Round 2: what the per-step timing events cost.  c2 pipelined and serial with
# no step events (HVWS_STEP_EVENTS=0) against the default, tail placement both
# ways, and kernel traces with events off.
set -u
S=scripts/gpu_step.sh
TAG=${1:-r2i}
export TMPDIR=/tmp
rm -f gpurun_out/.stop
B="python3 bench.py --steps 200 --warmup 10 --cpu-seconds 0 --host-gib 0 --no-tx --config c2"
for rep in 1 2; do
  for t in 0 1; do
    HVWS_TAIL=$t HVWS_STEP_EVENTS=0 $S bench_${TAG}_c2_ev0_t${t}_$rep 200 $B
    HVWS_TAIL=$t $S bench_${TAG}_c2_evd_t${t}_$rep 200 $B
  done
done
HVWS_STEP_EVENTS=0 $S bench_${TAG}_c2_ev0_serial 200 $B --serial
HVWS_TAIL=0 HVWS_STEP_EVENTS=0 $S trace_${TAG}_c2_t0 300 rocprofv3 --kernel-trace -d gpurun_out/trace_${TAG}_c2_t0 -o run --output-format csv -- python3 bench.py --config c2 --steps 20 --warmup 5 --cpu-seconds 0 --host-gib 0 --no-tx
HVWS_TAIL=1 HVWS_STEP_EVENTS=0 $S trace_${TAG}_c2_t1 300 rocprofv3 --kernel-trace -d gpurun_out/trace_${TAG}_c2_t1 -o run --output-format csv -- python3 bench.py --config c2 --steps 20 --warmup 5 --cpu-seconds 0 --host-gib 0 --no-tx
