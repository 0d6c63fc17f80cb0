# round 3: PMC counters for k_fused vs k_unmask at c2 (serial steps, probe script)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r3o
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM --output-format csv -d $R/gpurun_out/r3o/p1 -o p1 -- python3 $R/scripts/probe/fused_kernel.py c2 4096 > $R/gpurun_out/r3o/p1.log 2>&1 || { echo p1 failed; tail -5 $R/gpurun_out/r3o/p1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE WRITE_SIZE --output-format csv -d $R/gpurun_out/r3o/p2 -o p2 -- python3 $R/scripts/probe/fused_kernel.py c2 4096 > $R/gpurun_out/r3o/p2.log 2>&1 || { echo p2 failed; tail -5 $R/gpurun_out/r3o/p2.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SMEM SQ_WAIT_ANY SQ_INST_CYCLES_VMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY --output-format csv -d $R/gpurun_out/r3o/p3 -o p3 -- python3 $R/scripts/probe/fused_kernel.py c2 4096 > $R/gpurun_out/r3o/p3.log 2>&1 || { echo p3 failed; tail -5 $R/gpurun_out/r3o/p3.log; exit 1; }
ls $R/gpurun_out/r3o/p1 $R/gpurun_out/r3o/p2
