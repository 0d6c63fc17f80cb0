#!/bin/bash
# r6y2: the general ASan mode again with its result flushed before the exit
# handlers (r6y lost it to an exit-time CHECK failure in ASan's device
# allocator inside the HIP runtime's finalizer), and the same mode with the
# resident worker off, to see whether the exit failure depends on it.
set -u
S=scripts/gpu_step.sh
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
rm -f gpurun_out/.stop
make -C libhv_amd/csrc asan -j16 > gpurun_out/asan_build_r6y2.log 2>&1 && make -C tests/csrc asan >> gpurun_out/asan_build_r6y2.log 2>&1 || { echo "asan build failed"; tail -20 gpurun_out/asan_build_r6y2.log; exit 1; }
export ASAN_OPTIONS=detect_leaks=0
timeout -k 10 600 build/asan/asan_driver > gpurun_out/asan_all_r6y2.log 2>&1; echo "rc=$?"; head -3 gpurun_out/asan_all_r6y2.log
HVWS_DOOR=0 timeout -k 10 600 build/asan/asan_driver > gpurun_out/asan_all_nodoor_r6y2.log 2>&1; echo "rc=$?"; head -3 gpurun_out/asan_all_nodoor_r6y2.log
exit 0
