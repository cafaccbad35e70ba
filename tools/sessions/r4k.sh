#!/bin/bash
# r4 session k: fp64 'T' 16384^2 256^2 blocks over leading-dimension paddings (elements)
set -o pipefail
O=gpurun_out/r4k
mkdir -p $O
for pad in 0 2 4 6 8 10 12 14 16 24 32 48 64 96 128 192 256 512 1024 2048; do
  COSTA_PROBE_LDPAD=$pad timeout -k 10 200 python3 tools/order_probe.py f64 16384 256 0.0 10 >> $O/ldpad.txt 2>> $O/ldpad.err || exit 1
done
for pad in 0 8 16 32 64; do
  COSTA_PROBE_LDPAD=$pad timeout -k 10 200 python3 tools/order_probe.py f32 16384 256 0.0 10 >> $O/ldpad.txt 2>> $O/ldpad.err || exit 1
done
