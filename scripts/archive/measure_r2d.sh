#!/bin/bash
# Round 2: parity after the k_pscan cap fix (one-launch scan opt-in), then
# c2 step time with fewer timing markers (HVWS_STEP_EVENTS 2/1/0), pipelined
# and serial, and the one-launch scan on (fixed) for the record.
set -u
S=scripts/gpu_step.sh
TAG=${1:-r2d}
export TMPDIR=/tmp
rm -f gpurun_out/.stop
$S parity_$TAG 500 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread
B="python3 bench.py --steps 40 --warmup 5 --cpu-seconds 0 --host-gib 0 --no-tx --config c2"
for ev in 2 1 0; do
  HVWS_STEP_EVENTS=$ev $S bench_${TAG}_c2_ev$ev 200 $B
  HVWS_STEP_EVENTS=$ev $S bench_${TAG}_c2_ev${ev}_serial 200 $B --serial
done
HVWS_PSCAN=1 $S bench_${TAG}_c2_pscan 200 $B
HVWS_PSCAN=1 $S bench_${TAG}_c2_pscan_serial 200 $B --serial
