#!/bin/bash
# r4 session zb: panel heights around the shipped 128 KiB for c128 32768^2 (alpha, beta)
set -o pipefail
O=gpurun_out/r4zb
mkdir -p $O
for rep in 1 2; do
for h in 0 6144 10240 12288; do
  echo -n "panel $h " >> $O/panels.txt
  COSTA_TUNING=1 COSTA_PANEL_ROWS=$h timeout -k 10 200 python3 tools/order_probe.py c128 32768 128 1.0 6 >> $O/panels.txt 2>> $O/err.txt || exit 1
done
done
