#!/bin/bash
# r5 session a: staging of the full transposing sub-tiles (COSTA_TR_STAGE tuning builds):
# 1 LDS-DMA, 2 LDS-DMA in two row halves, 3 LDS-DMA with wave-contiguous columns, 4 register
# staging in two halves, 5 register staging with wave-contiguous columns; against the shipped
# build, alternating, each run verified (bench.py)
set -o pipefail
O=gpurun_out/r5a
mkdir -p $O
timeout -k 10 900 python3 tools/ab_bench.py $O 3 shipped: \
  st1:COSTA_LIB=gpuvar/st1/lib/libcosta_amd.so st2:COSTA_LIB=gpuvar/st2/lib/libcosta_amd.so \
  st3:COSTA_LIB=gpuvar/st3/lib/libcosta_amd.so st4:COSTA_LIB=gpuvar/st4/lib/libcosta_amd.so \
  st5:COSTA_LIB=gpuvar/st5/lib/libcosta_amd.so \
  -- --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --no-extra
