#!/bin/bash
# pack / unpack lists of small-block transposes (every tile through the loopback exchange) with
# and without merging
set -o pipefail
O=gpurun_out/${1:-mergelb}; mkdir -p $O
for m in 1 0; do
  for cfg in "f32 16384 24 0" "f64 16384 24 1" "f64 16384 256 0"; do
    COSTA_LOOPBACK=1 COSTA_MERGE=$m timeout -k 10 120 python3 tools/order_probe.py $cfg 10 2>/dev/null | sed "s/^/merge=$m /" >> $O/lb.txt || exit 1
  done
done
