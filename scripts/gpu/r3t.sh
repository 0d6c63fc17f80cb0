#!/bin/bash
# round 3: windowed sieve geometry sweep at c4 one stream (hops x window), and
# a kernel trace at hops 256
set -u
S=scripts/gpu_step.sh
TAG=${1:-r3u}
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
rm -f gpurun_out/.stop
B="python3 bench.py --config c4 --segments 1 --steps 20 --warmup 3 --cpu-seconds 0 --host-gib 0 --no-tx --feed-conns 0 --dropin-reads 0"
for hw in 64:0 128:0 256:0 384:0 512:0 768:0 256:524288 512:524288 128:0 256:0 384:0 512:0; do
  h=${hw%%:*}; w=${hw##*:}
  [ "$w" = 0 ] && unset HVWS_SIEVE_WINDOW || export HVWS_SIEVE_WINDOW=$w
  HVWS_SIEVE_HOPS=$h $S c4s1_h${h}_w${w}_$TAG 200 $B
  grep -h '"metric"' gpurun_out/c4s1_h${h}_w${w}_$TAG.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('hops=$h win=$w', d['value'], d['ms_per_step'], d['unmask_ms_mean'], d.get('roofline',{}).get('frac'))" || true
done
unset HVWS_SIEVE_WINDOW
HVWS_SIEVE_HOPS=384 $S trace_c4s1_h384_$TAG 300 rocprofv3 --kernel-trace --stats -d gpurun_out/trace_c4s1_h384_$TAG -o run --output-format csv -- $B
