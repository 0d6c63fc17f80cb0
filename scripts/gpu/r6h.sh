#!/bin/bash
# r6h: transmit with its default XCD runs (lean 8, 64x4 2) -- tests, speed
# against runs of 1 (interleaved), DRAM-side reads; door tests (record-major XOR back).
set -u
S=scripts/gpu_step.sh
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
rm -f gpurun_out/.stop
$S pytest_txdoor_r6h 400 python -u -m pytest tests/test_gpu_tx.py tests/test_gpu_door.py -x -q --timeout 120 --timeout-method thread
[ -f gpurun_out/.stop ] && exit 1
for i in 1 2 3; do
  for xg in d 1; do
    if [ $xg = d ]; then E=""; else E="build_xgroup=1"; fi
    HVWS_EXPERIMENT=$E CONFIG=c3 REPS=5 $S tx_c3_${xg}_${i}_r6h 300 python3 scripts/bench_tx.py
    [ -f gpurun_out/.stop ] && exit 1
    HVWS_EXPERIMENT=$E CONFIG=c2 REPS=5 $S tx_c2_${xg}_${i}_r6h 300 python3 scripts/bench_tx.py
    [ -f gpurun_out/.stop ] && exit 1
  done
done
for cfg in c2 c3; do
  CONFIG=$cfg REPS=2 $S pmc_rd_tx_${cfg}_r6h 300 timeout -s KILL 280 rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_32B_sum TCC_EA0_RDREQ_sum --output-format csv -d gpurun_out/r6h_pmc_rd_tx_${cfg} -o p -- python3 scripts/bench_tx.py
  [ -f gpurun_out/.stop ] && exit 1
  CONFIG=$cfg REPS=2 $S pmc_wr_tx_${cfg}_r6h 300 timeout -s KILL 280 rocprofv3 --pmc WRITE_SIZE TCC_EA0_WRREQ_WRITE_DRAM_32B_sum --output-format csv -d gpurun_out/r6h_pmc_wr_tx_${cfg} -o p -- python3 scripts/bench_tx.py
  [ -f gpurun_out/.stop ] && exit 1
done
exit 0
