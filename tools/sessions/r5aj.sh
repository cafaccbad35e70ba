#!/bin/bash
# r5 session aj: the wavefront copy path with fewer bytes a lane per pass (tuning builds of
# engine.hpp tiny_copy_lane_bytes: 32, 16 against 64), cfg 5 'N' with every op on the wavefront
# path (COSTA_CBLOCK=0, the multi-rank pack lists' situation) and as shipped
set -o pipefail
O=gpurun_out/r5aj
mkdir -p $O
V=gpuvar
E=COSTA_TUNING=1,COSTA_CBLOCK=0
timeout -k 10 400 python3 tools/ab_bench.py $O/c5N_wave 2 shipped:$E lb32:$E,COSTA_LIB=$V/lb32/lib/libcosta_amd.so \
  lb16:$E,COSTA_LIB=$V/lb16/lib/libcosta_amd.so \
  -- --workload cfg5 --cfg5-op N --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --no-extra || exit 1
