#!/bin/bash
# pack / unpack lists of cfg 2's layout (loopback exchange, one round: kernels alone) under the
# large-shape sub-tile orders (COSTA_LARGE_SORT 0..3), twice
set -o pipefail
O=gpurun_out/${1:-packsort}; mkdir -p $O
for rep in 1 2; do
  for m in 3 0 1 2; do
    COSTA_LARGE_SORT=$m COSTA_LOOPBACK=1 COSTA_EXCHANGE_ROUNDS=1 timeout -k 10 120 python3 tools/order_probe.py f64 16384 256 0 10 2>/dev/null | grep "^f64" | sed "s/^/sort=$m /" >> $O/ps.txt || exit 1
    COSTA_LARGE_SORT=$m COSTA_LOOPBACK=1 COSTA_EXCHANGE_ROUNDS=1 timeout -k 10 120 python3 tools/order_probe.py f64 16384 128 1 10 2>/dev/null | grep "^f64" | sed "s/^/sort=$m /" >> $O/ps.txt || exit 1
  done
done
