#!/bin/bash
# r4 session l: transposes into destination columns 16-byte aligned but off the 64-byte granule
# grid, on the large shape (shipped) or the skew shape (COSTA_SKEW_GRANULE=1)
set -o pipefail
O=gpurun_out/r4l
mkdir -p $O
for a in "f64 16384 256 0.0" "f64 16384 128 1.0" "f32 16384 256 0.0"; do
  for pad in 0 2 4 8 16 24 64; do
    for e in 0 1; do
      echo -n "granule=$e " >> $O/ldpad.txt
      COSTA_TUNING=1 COSTA_SKEW_GRANULE=$e COSTA_PROBE_LDPAD=$pad timeout -k 10 200 python3 tools/order_probe.py $a 10 >> $O/ldpad.txt 2>> $O/ldpad.err || exit 1
    done
  done
done
for pad in 0 2 8 16; do
  COSTA_PROBE_OP=N COSTA_PROBE_LDPAD=$pad timeout -k 10 200 python3 tools/order_probe.py f64 16384 256 0.0 10 >> $O/copy_ldpad.txt 2>> $O/ldpad.err || exit 1
done
