#!/bin/bash
# r5 session ak: cfg 5 'N' destination-block groups in 4-group XCD chunks (tuning build
# gpuvar/nxk) with destination order and with source order (COSTA_CBLOCK_ORDER=1: groups reading
# neighbouring source lines consecutive, hence on one XCD), against the shipped round-robin
set -o pipefail
O=gpurun_out/r5ak
mkdir -p $O
V=gpuvar
timeout -k 10 400 python3 tools/ab_bench.py $O/c5N 2 shipped: src:COSTA_TUNING=1,COSTA_CBLOCK_ORDER=1 \
  nxk:COSTA_LIB=$V/nxk/lib/libcosta_amd.so nxk_src:COSTA_TUNING=1,COSTA_CBLOCK_ORDER=1,COSTA_LIB=$V/nxk/lib/libcosta_amd.so \
  -- --workload cfg5 --cfg5-op N --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --no-extra || exit 1
timeout -k 10 400 python3 tools/ab_bench.py $O/c5T 2 shipped: src:COSTA_TUNING=1,COSTA_CBLOCK_ORDER=1 \
  -- --workload cfg5 --cfg5-op T --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --no-extra || exit 1
