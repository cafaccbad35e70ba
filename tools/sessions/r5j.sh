#!/bin/bash
# r5 session j: builds side by side on the same buffers (tools/libs_probe.py): the shipped kernel,
# LDS-DMA staging (st1), one-column stores (st6), column-pair store order (st7), 1024 threads per
# 64 x 128 sub-tile, on 8 pairs (fast and slow destination placements alike)
set -o pipefail
O=gpurun_out/r5j
mkdir -p $O
V=gpuvar
timeout -k 10 300 python3 tools/libs_probe.py 8 shipped=costa_amd/lib/libcosta_amd.so st1=$V/st1/lib/libcosta_amd.so \
  st6=$V/st6/lib/libcosta_amd.so st7=$V/st7/lib/libcosta_amd.so t1024=$V/f64x128t1024/lib/libcosta_amd.so \
  > $O/libs.txt 2>&1 || exit 1
