#!/bin/bash
# r4 session x: 1 KiB segments from the column start against address-aligned 1 KiB windows
set -o pipefail
O=gpurun_out/r4x
mkdir -p $O
timeout -k 10 120 tools/stride_probe windows > $O/windows.txt 2>&1 || exit 1
# fp64 16384^2 'T' at a 384 KiB column stride (lld 49152) under other sub-tile orders
for e in "" "COSTA_LARGE_SORT=1" "COSTA_PANEL_ROWS=4096" "COSTA_PANEL_ROWS=8192" "COSTA_PANEL_ROWS=-1"; do
  echo -n "[$e] " >> $O/ld384_orders.txt
  env COSTA_TUNING=1 $e COSTA_PROBE_LDPAD=32768 timeout -k 10 200 python3 tools/order_probe.py f64 16384 256 0.0 10 >> $O/ld384_orders.txt 2>> $O/err.txt || exit 1
done
