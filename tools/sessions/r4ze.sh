#!/bin/bash
# r4 session ze: inside each destination panel, B column bands walked together (COSTA_PANEL_BANDS)
set -o pipefail
O=gpurun_out/r4ze
mkdir -p $O
for rep in 1 2; do
  for b in 0 4 8 16 32; do
    echo -n "bands $b " >> $O/bands.txt
    COSTA_TUNING=1 COSTA_PANEL_BANDS=$b timeout -k 10 200 python3 tools/order_probe.py c128 32768 128 1.0 6 >> $O/bands.txt 2>> $O/err.txt || exit 1
  done
done
for b in 0 8 16; do
  echo -n "bands $b " >> $O/bands.txt
  COSTA_TUNING=1 COSTA_PANEL_BANDS=$b timeout -k 10 200 python3 tools/order_probe.py c128 16384 128 1.0 10 >> $O/bands.txt 2>> $O/err.txt || exit 1
  echo -n "bands $b " >> $O/bands.txt
  COSTA_TUNING=1 COSTA_PANEL_BANDS=$b timeout -k 10 200 python3 tools/order_probe.py f64 32768 256 0.0 10 >> $O/bands.txt 2>> $O/err.txt || exit 1
  echo -n "bands $b " >> $O/bands.txt
  COSTA_TUNING=1 COSTA_PANEL_BANDS=$b timeout -k 10 200 python3 tools/order_probe.py f64 16384 256 0.0 10 >> $O/bands.txt 2>> $O/err.txt || exit 1
done
