#!/bin/bash
# r4 session j: does a power-of-two leading dimension cost the transposes?  (ld padding)
set -o pipefail
O=gpurun_out/r4j
mkdir -p $O
for a in "c128 32768 128 1.0" "c128 16384 128 1.0" "f64 16384 256 0.0" "f64 32768 128 1.0"; do
  for pad in 0 8 32 256; do
    COSTA_PROBE_LDPAD=$pad timeout -k 10 200 python3 tools/order_probe.py $a 10 >> $O/ldpad.txt 2>> $O/ldpad.err || exit 1
  done
done
