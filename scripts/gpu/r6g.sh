#!/bin/bash
# r6g: the worker read's chunk-major XOR -- door, feed and parity tests, then
# the drop-in latency and the phase stamps against the previous build
# (build/ab/libhvws_head.so), interleaved.
set -u
S=scripts/gpu_step.sh
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
rm -f gpurun_out/.stop
$S pytest_door_r6g 400 python -u -m pytest tests/test_gpu_door.py tests/test_gpu_feed_many.py tests/test_gpu_validate.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread
[ -f gpurun_out/.stop ] && exit 1
for i in 1 2; do
  $S dropin_new${i}_r6g 200 python3 scripts/bench_dropin.py
  [ -f gpurun_out/.stop ] && exit 1
  HVWS_LIB=build/ab/libhvws_head.so $S dropin_old${i}_r6g 200 python3 scripts/bench_dropin.py
  [ -f gpurun_out/.stop ] && exit 1
done
HVWS_EXPERIMENT=feed_times=1 $S dph_new_r6g 200 python3 scripts/probe/door_phases.py 4000
[ -f gpurun_out/.stop ] && exit 1
HVWS_LIB=build/ab/libhvws_head.so HVWS_EXPERIMENT=feed_times=1 $S dph_old_r6g 200 python3 scripts/probe/door_phases.py 4000
# transmit: tile runs per XCD (build_xgroup) -- correctness, speed, DRAM-side reads
[ -f gpurun_out/.stop ] && exit 1
HVWS_EXPERIMENT=build_xgroup=4 $S pytest_tx_xg4_r6g 300 python -u -m pytest tests/test_gpu_tx.py -x -q --timeout 120 --timeout-method thread
[ -f gpurun_out/.stop ] && exit 1
for cfg in c2 c3; do
  for xg in 1 4 8 2 1 4; do
    HVWS_EXPERIMENT=build_xgroup=$xg CONFIG=$cfg REPS=5 $S tx_${cfg}_xg${xg}_r6g 300 python3 scripts/bench_tx.py
    [ -f gpurun_out/.stop ] && exit 1
  done
done
for cfg in c2 c3; do
  for xg in 1 4 8; do
    HVWS_EXPERIMENT=build_xgroup=$xg CONFIG=$cfg REPS=2 $S pmc_tx_${cfg}_xg${xg}_r6g 300 timeout -s KILL 280 rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_32B_sum TCC_EA0_RDREQ_sum --output-format csv -d gpurun_out/r6g_pmc_tx_${cfg}_xg${xg} -o p -- python3 scripts/bench_tx.py
    [ -f gpurun_out/.stop ] && exit 1
  done
done
exit 0
