#!/bin/bash
# round 3: windowed sieve, wave-per-node emit, 256-thread LDS doubling --
# sieve parity + full-size c4, then hops 192-384 twice and a trace at 256
set -u
S=scripts/gpu_step.sh
TAG=${1:-r3w}
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
rm -f gpurun_out/.stop
$S pytest_sieve_$TAG 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "sieve"
grep -q " passed" gpurun_out/pytest_sieve_$TAG.log && ! grep -q "failed" gpurun_out/pytest_sieve_$TAG.log || { echo "sieve tests not green"; exit 1; }
$S pytest_c4_$TAG 300 python -u -m pytest tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread -k "config4"
B="python3 bench.py --config c4 --segments 1 --steps 20 --warmup 3 --cpu-seconds 0 --host-gib 0 --no-tx --feed-conns 0 --dropin-reads 0"
for h in 64 192 256 320 384 192 256 320 384; do
  HVWS_SIEVE_HOPS=$h $S c4s1_h${h}_$TAG 200 $B
  grep -h '"metric"' gpurun_out/c4s1_h${h}_$TAG.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('hops=$h', d['value'], d['ms_per_step'], d['unmask_ms_mean'], d.get('roofline',{}).get('frac'))" || true
done
$S trace_c4s1_$TAG 300 rocprofv3 --kernel-trace --stats -d gpurun_out/trace_c4s1_$TAG -o run --output-format csv -- $B
