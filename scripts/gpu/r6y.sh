#!/bin/bash
# r6y: the host code under AddressSanitizer (host side only; device code is
# untouched) after round 6's worker changes (its own HSA queue, the block
# poll's seq_tail, the one-writeback release): build the ASan library and
# driver on the box, then the worker's paths with a process exit ("door") and
# the general receive / transmit paths.
set -u
S=scripts/gpu_step.sh
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
rm -f gpurun_out/.stop
make -C libhv_amd/csrc asan -j16 > gpurun_out/asan_build_r6y.log 2>&1 && make -C oracle > /dev/null 2>&1; make -C tests/csrc asan >> gpurun_out/asan_build_r6y.log 2>&1 || { echo "asan build failed"; tail -20 gpurun_out/asan_build_r6y.log; exit 1; }
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=0
$S asan_door_r6y 300 build/asan/asan_driver door
[ -f gpurun_out/.stop ] && exit 1
$S asan_all_r6y 600 build/asan/asan_driver
exit 0
