#!/bin/bash
# r6f: (1) drop-in latency, the worker on its HSA queue against the round-5
# CU-masked stream build (build/ab), interleaved; (2) the worker's phase
# stamps; (3) HBM bytes of the transmit kernels from the DRAM-side 32-byte
# counters beside the FETCH_SIZE correction (c2, c3), and k_unmask at c2 as
# the calibration (separate --pmc passes).
set -u
S=scripts/gpu_step.sh
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
rm -f gpurun_out/.stop
$S pytest_gpu_r6f 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
[ -f gpurun_out/.stop ] && exit 1
for i in 1 2; do
  $S dropin_new${i}_r6f 200 python3 scripts/bench_dropin.py
  [ -f gpurun_out/.stop ] && exit 1
  HVWS_LIB=build/ab/libhvws_cumask.so $S dropin_old${i}_r6f 200 python3 scripts/bench_dropin.py
  [ -f gpurun_out/.stop ] && exit 1
done
HVWS_EXPERIMENT=feed_times=1 $S dph_r6f 200 python3 scripts/probe/door_phases.py 4000
[ -f gpurun_out/.stop ] && exit 1
for cfg in c2 c3; do
  for pass in "TCC_EA0_RDREQ_DRAM_32B_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" "FETCH_SIZE TCC_BUBBLE_sum" "WRITE_SIZE TCC_EA0_WRREQ_WRITE_DRAM_32B_sum"; do
    tag=$(echo $pass | cut -c1-12 | tr -dc 'A-Za-z0-9_')
    CONFIG=$cfg REPS=2 $S pmc_${tag}_tx_${cfg}_r6f 300 timeout -s KILL 280 rocprofv3 --pmc $pass --output-format csv -d gpurun_out/r6f_pmc_tx_${cfg}_${tag} -o p -- python3 scripts/bench_tx.py
    [ -f gpurun_out/.stop ] && exit 1
  done
done
B="--config c2 --steps 4 --warmup 1 --no-tx --feed-conns 0 --dropin-reads 0 --host-gib 0 --cpu-seconds 0"
for pass in "TCC_EA0_RDREQ_DRAM_32B_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" "FETCH_SIZE TCC_BUBBLE_sum" "WRITE_SIZE TCC_EA0_WRREQ_WRITE_DRAM_32B_sum"; do
  tag=$(echo $pass | cut -c1-12 | tr -dc 'A-Za-z0-9_')
  HVWS_RUN=0 $S pmc_${tag}_c2_r6f 200 timeout -s KILL 180 rocprofv3 --pmc $pass --output-format csv -d gpurun_out/r6f_pmc_c2_${tag} -o p -- python3 bench.py $B
  [ -f gpurun_out/.stop ] && exit 1
done
exit 0
