#!/bin/bash
# r5 session v: fp64 copy shapes with fewer loads a thread in flight (tuning builds of
# tile_kernels.hip COSTA_F64_COPY: 1 = 1024 threads x 1 load, 2 = 512 x 2, 3 = 256 x 4, all on
# 128 x 16 sub-tiles) against the shipped 256 threads x 32 loads (128 x 128), cfg 3's copy slice
set -o pipefail
O=gpurun_out/r5v
mkdir -p $O
V=gpuvar
timeout -k 10 900 python3 tools/ab_bench.py $O/c3 2 shipped: cp1:COSTA_LIB=$V/cp1/lib/libcosta_amd.so \
  cp2:COSTA_LIB=$V/cp2/lib/libcosta_amd.so cp3:COSTA_LIB=$V/cp3/lib/libcosta_amd.so \
  -- --workload cfg3 --steps 10 --warmup 2 --no-cpu-baseline --no-e2e --no-extra || exit 1
