#!/bin/bash
# copy ('N') lists of block-cyclic layouts: local, and pack / unpack through the loopback exchange
# (one round), under large-shape orders COSTA_LARGE_SORT 3 (default) / 2 (by destination), twice
set -o pipefail
O=gpurun_out/${1:-packsort2}; mkdir -p $O
for rep in 1 2; do
  for m in 3 2; do
    for cfg in "f64 16384 128 0" "f64 16384 256 0" "c128 16384 128 1" "f32 16384 256 0"; do
      COSTA_PROBE_OP=N COSTA_LARGE_SORT=$m timeout -k 10 120 python3 tools/order_probe.py $cfg 10 2>/dev/null | grep -v "^ *$" | sed "s/^/N local sort=$m /" >> $O/ps.txt || exit 1
      COSTA_PROBE_OP=N COSTA_LARGE_SORT=$m COSTA_LOOPBACK=1 COSTA_EXCHANGE_ROUNDS=1 timeout -k 10 120 python3 tools/order_probe.py $cfg 10 2>/dev/null | grep "^[fc]" | sed "s/^/N loopback sort=$m /" >> $O/ps.txt || exit 1
    done
    COSTA_LARGE_SORT=$m COSTA_LOOPBACK=1 COSTA_EXCHANGE_ROUNDS=1 timeout -k 10 120 python3 tools/order_probe.py c128 16384 128 1 10 2>/dev/null | grep "^c" | sed "s/^/T loopback sort=$m /" >> $O/ps.txt || exit 1
  done
done
