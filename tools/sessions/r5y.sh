#!/bin/bash
# r5 session y: c128's square transposing sub-tile (64 x 64, cfg 4) with 512 / 1024 threads (8 / 4
# loads a thread) against the shipped 256 (16 loads), cfg 4's 32768^2 slice, alternating
set -o pipefail
O=gpurun_out/r5y
mkdir -p $O
V=gpuvar
timeout -k 10 1000 python3 tools/ab_bench.py $O/c4 2 shipped: sq512:COSTA_LIB=$V/sq512/lib/libcosta_amd.so \
  sq1024:COSTA_LIB=$V/sq1024/lib/libcosta_amd.so \
  -- --workload cfg4 --edge 32768 --steps 5 --warmup 2 --no-cpu-baseline --no-e2e --no-extra || exit 1
