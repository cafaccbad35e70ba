#!/bin/bash
# r4 session p: destination-ordered sub-tiles walked in panels of H target rows (COSTA_PANEL_ROWS)
set -o pipefail
O=gpurun_out/r4p
mkdir -p $O
for a in "c128 32768 128 1.0" "c128 16384 128 1.0" "f64 16384 256 0.0" "f64 32768 128 1.0"; do
  for h in 0 2048 4096 8192 16384; do
    echo -n "H=$h " >> $O/panels.txt
    COSTA_TUNING=1 COSTA_PANEL_ROWS=$h timeout -k 10 200 python3 tools/order_probe.py $a 10 >> $O/panels.txt 2>> $O/panels.err || exit 1
  done
done
