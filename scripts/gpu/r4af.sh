#!/bin/bash
# round 4: k_build variant 7 (lean, LDS-DMA span staging, no streaming path,
# lane id recomputed: 64 VGPRs without spills = 8 waves per SIMD) and the
# keys loaded with the records (no second round trip) against 0 / 5 / 6;
# the frame sieve's tile prefetch now overlapping (the halo load under a
# lane mask had forced a wait for it): c4 one stream, default vs mode 4 (no
# prefetch), steps and kernel trace
set -u
S=scripts/gpu_step.sh
TAG=${1:-r4af}
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONFAULTHANDLER=1
rm -f gpurun_out/.stop
$S pytest_tx_$TAG 400 python -u -m pytest tests/test_gpu_tx.py -x -q --timeout 120 --timeout-method thread
[ -f gpurun_out/.stop ] && exit 1
HVWS_BUILD=7 $S pytest_tx_b7_$TAG 400 python -u -m pytest tests/test_gpu_tx.py -x -q --timeout 120 --timeout-method thread -k "not every_geometry and not by_frame_size"
[ -f gpurun_out/.stop ] && exit 1
$S pytest_sieve_$TAG 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 120 --timeout-method thread -k "sieve or c4 or single or stream"
[ -f gpurun_out/.stop ] && exit 1
for rep in 1 2; do
  for cfg in c2 c3 c4; do
    for v in 0 5 6 7; do
      HVWS_BUILD=$v CONFIG=$cfg $S tx_${cfg}_b${v}_${rep}_$TAG 200 python3 scripts/bench_tx.py
      [ -f gpurun_out/.stop ] && exit 1
    done
  done
done
L="--steps 40 --warmup 5 --cpu-seconds 0 --host-gib 0 --no-tx --feed-conns 0 --dropin-reads 0"
for rep in 1 2; do
  $S c4s1_m0_${rep}_$TAG 200 python3 bench.py --config c4 --segments 1 $L
  [ -f gpurun_out/.stop ] && exit 1
  HVWS_SIEVE_MODE=4 $S c4s1_m4_${rep}_$TAG 200 python3 bench.py --config c4 --segments 1 $L
  [ -f gpurun_out/.stop ] && exit 1
done
for m in 0 4; do
  HVWS_DOOR_POOL=0 HVWS_SIEVE_MODE=$m $S trace_c4s1_m${m}_$TAG 300 rocprofv3 --kernel-trace --stats -d gpurun_out/trace_c4s1_m${m}_$TAG -o run --output-format csv -- python3 bench.py --config c4 --segments 1 $L
  [ -f gpurun_out/.stop ] && exit 1
done
exit 0
