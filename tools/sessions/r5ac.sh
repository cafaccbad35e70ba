#!/bin/bash
# r5 session ac: destination-block groups in chunks of k consecutive groups per XCD (the 8 XCDs on
# 8 adjacent chunks; tuning builds gpuvar/xk{2,4,16}, tile_kernels.hip COSTA_CB_XK, 'T' and 'N'
# alike) against the shipped order (XCD-contiguous slices for 'T', round-robin for 'N'), cfg 5
set -o pipefail
O=gpurun_out/r5ac
mkdir -p $O
V=gpuvar
L="shipped: xk2:COSTA_LIB=$V/xk2/lib/libcosta_amd.so xk4:COSTA_LIB=$V/xk4/lib/libcosta_amd.so xk16:COSTA_LIB=$V/xk16/lib/libcosta_amd.so"
timeout -k 10 400 python3 tools/ab_bench.py $O/c5T 2 $L \
  -- --workload cfg5 --cfg5-op T --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --no-extra || exit 1
timeout -k 10 400 python3 tools/ab_bench.py $O/c5N 2 $L \
  -- --workload cfg5 --cfg5-op N --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --no-extra || exit 1
