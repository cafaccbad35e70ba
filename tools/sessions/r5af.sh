#!/bin/bash
# r5 session af: the wavefront path's XCD mapping -- chunks of k consecutive workgroups per XCD
# (tuning builds gpuvar/ty{4,16,64}, tile_kernels.hip COSTA_TINY_XK) against the shipped
# contiguous slice per XCD, on cfg 5 with the destination-block groups off (COSTA_CBLOCK=0: every
# op on the wavefront path, as in the pack lists of a multi-rank cfg 5)
set -o pipefail
O=gpurun_out/r5af
mkdir -p $O
V=gpuvar
E=COSTA_TUNING=1,COSTA_CBLOCK=0
L="shipped:$E ty4:$E,COSTA_LIB=$V/ty4/lib/libcosta_amd.so ty16:$E,COSTA_LIB=$V/ty16/lib/libcosta_amd.so ty64:$E,COSTA_LIB=$V/ty64/lib/libcosta_amd.so"
timeout -k 10 400 python3 tools/ab_bench.py $O/c5T 2 $L \
  -- --workload cfg5 --cfg5-op T --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --no-extra || exit 1
timeout -k 10 400 python3 tools/ab_bench.py $O/c5N 2 $L \
  -- --workload cfg5 --cfg5-op N --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --no-extra || exit 1
