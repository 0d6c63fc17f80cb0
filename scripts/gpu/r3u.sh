#!/bin/bash
# round 3: windowed sieve with stored walk offsets and one-launch doubling --
# sieve parity subset, then the geometry sweep (r3t.sh) under tag r3u
set -u
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
rm -f gpurun_out/.stop
scripts/gpu_step.sh pytest_sieve_r3u 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "sieve"
grep -q " passed" gpurun_out/pytest_sieve_r3u.log && ! grep -q "failed" gpurun_out/pytest_sieve_r3u.log || { echo "sieve tests not green"; exit 1; }
scripts/gpu_step.sh pytest_c4_r3u 300 python -u -m pytest tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread -k "config4"
bash scripts/gpu/r3t.sh r3u
