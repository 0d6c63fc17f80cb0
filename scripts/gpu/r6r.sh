#!/bin/bash
# r6r: two ranks rehearsed on one card (HVWS_BENCH_DEVICE=0), through bench.py's
# own launcher and through torch.distributed.run: the per-rank unmask time,
# roofline fraction and stream ceiling in timing.per_rank on hardware.
set -u
S=scripts/gpu_step.sh
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
rm -f gpurun_out/.stop
A="--gpus 2 --steps 5 --warmup 2 --no-tx --feed-conns 0 --dropin-reads 0 --host-gib 0 --cpu-seconds 0"
HVWS_BENCH_DEVICE=0 $S rehearsal_launcher_r6r 400 python3 bench.py $A
[ -f gpurun_out/.stop ] && exit 1
HVWS_BENCH_DEVICE=0 $S rehearsal_torchrun_r6r 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py $A
exit 0
