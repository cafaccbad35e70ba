#!/bin/bash
# r5 session h: which buffer's placement decides the headline's mode (4 A x 4 C buffers, every
# combination), and the 8-pair distribution of other sub-tile shapes / staging (tuning builds):
# fp64 128 x 64 (1 KiB source segments), 128 x 128 with 1024 threads, 64 x 128 with 1024 threads,
# LDS-DMA staging
set -o pipefail
O=gpurun_out/r5h
mkdir -p $O
timeout -k 10 200 python3 tools/pairs_probe.py cross 4 > $O/cross.txt 2>&1 || exit 1
timeout -k 10 150 python3 tools/pairs_probe.py 8 1 > $O/pairs_shipped.txt 2>&1 || exit 1
for v in f128x64 f128x128 f64x128t1024 st1; do
  COSTA_LIB=gpuvar/$v/lib/libcosta_amd.so timeout -k 10 150 python3 tools/pairs_probe.py 8 1 > $O/pairs_$v.txt 2>&1 || exit 1
done
