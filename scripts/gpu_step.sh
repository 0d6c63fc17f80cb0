#!/bin/bash
# Run one GPU step under its own time limit; record its status; refuse to go
# on after any failure (a crash, a time limit, a failed test -- which may be a
# GPU fault reported as an exception) so no further GPU work starts in the
# same gpurun call.
#   scripts/gpu_step.sh NAME SECONDS cmd...
name=$1; secs=$2; shift 2
mkdir -p gpurun_out
if [ -f gpurun_out/.stop ]; then echo "[$name] skipped (earlier crash)"; exit 0; fi
echo "[$name] start $(date +%T)"
timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
rc=$?
echo "[$name] rc=$rc $(date +%T)"
tail -5 "gpurun_out/$name.log"
[ $rc -ne 0 ] && touch gpurun_out/.stop
exit 0
