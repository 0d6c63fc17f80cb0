#!/bin/bash
# Pipelined-step experiment: capped unmask grid (HVWS_PIPE_GRID) so the next
# batch's discovery can co-reside; c2, c3, c4.
# (Experiment record: the capped grid lost 13-16 % of unmask throughput, so the
# HVWS_PIPE_GRID knob was removed afterwards; outputs in profiles/r1k_raw/.)
set -u
S=scripts/gpu_step.sh
TAG=${1:-r1k}
export TMPDIR=/tmp
for g in 0 1024 2048 3072; do
  HVWS_PIPE_GRID=$g $S bench_${TAG}_c2_g$g 200 python bench.py --config c2 --cpu-seconds 0 --host-gib 0 --no-tx
done
for g in 0 1024 2048; do
  HVWS_PIPE_GRID=$g $S bench_${TAG}_c3_g$g 300 python bench.py --cpu-seconds 0 --host-gib 0 --no-tx
done
for g in 0 2048; do
  HVWS_PIPE_GRID=$g $S bench_${TAG}_c4_g$g 200 python bench.py --config c4 --segments 1024 --cpu-seconds 0 --host-gib 0 --no-tx
done
