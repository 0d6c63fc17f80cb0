#!/bin/bash
# Event-loop threads on one GPU vs the reference on the same threads
# (scripts/feed_mt.cpp).  Builds the harness if needed; one JSON line per run.
set -e
[ -x build/feed_mt ] && [ build/feed_mt -nt scripts/feed_mt.cpp ] || /opt/rocm/bin/hipcc -O2 -std=c++17 -Iinclude scripts/feed_mt.cpp -Llibhv_amd -lhvws \
    -Wl,-rpath,'$ORIGIN/../libhv_amd' -ldl -lpthread -o build/feed_mt
MODES=${MODES:-gpu ref}
for C in ${CONNS:-256 1024}; do
  for T in ${THREADS:-1 2 4 8}; do
    for m in $MODES; do
      timeout -k 10 120 ./build/feed_mt $m $T $C 20
    done
  done
done
