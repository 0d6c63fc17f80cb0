#!/bin/bash
# Event-loop threads on one GPU vs the reference on the same threads
# (scripts/feed_mt.cpp).  Builds the harness if needed; one JSON line per run.
set -e
[ -x build/feed_mt ] || /opt/rocm/bin/hipcc -O2 -std=c++17 -Iinclude scripts/feed_mt.cpp -Llibhv_amd -lhvws \
    -Wl,-rpath,'$ORIGIN/../libhv_amd' -ldl -lpthread -o build/feed_mt
for C in 256 1024; do
  for T in 1 2 4 8; do
    timeout -k 10 120 ./build/feed_mt gpu $T $C 20
    timeout -k 10 120 ./build/feed_mt ref $T $C 20
  done
done
