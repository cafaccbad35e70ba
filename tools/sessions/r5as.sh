#!/bin/bash
# r5 session as: destination-block group budgets for the copy: 8 KiB / 32 KiB groups (tuning builds
# of engine.hpp kCblockChunks 2 / 8) against the shipped 16 KiB, cfg 5 'N' (and 'T' with the XCD
# chunks)
set -o pipefail
O=gpurun_out/r5as
mkdir -p $O
V=gpuvar
L="shipped: c2:COSTA_LIB=$V/cbc2/lib/libcosta_amd.so c8:COSTA_LIB=$V/cbc8/lib/libcosta_amd.so"
timeout -k 10 400 python3 tools/ab_bench.py $O/c5N 2 $L \
  -- --workload cfg5 --cfg5-op N --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --no-extra || exit 1
timeout -k 10 400 python3 tools/ab_bench.py $O/c5T 2 $L \
  -- --workload cfg5 --cfg5-op T --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --no-extra || exit 1
