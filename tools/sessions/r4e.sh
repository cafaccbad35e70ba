#!/bin/bash
# r4 session e: c128 'T' 128^2 blocks: square 64 x 64 sub-tiles x sub-tile orders
set -o pipefail
O=gpurun_out/r4e
mkdir -p $O
for n in 16384 32768; do
  for e in "" "COSTA_TUNING=1 COSTA_FORCE_SQ=1 COSTA_LARGE_SORT=2" "COSTA_TUNING=1 COSTA_FORCE_SQ=1" "COSTA_TUNING=1 COSTA_LARGE_SORT=2" "COSTA_TUNING=1 COSTA_FORCE_SQ=1 COSTA_LARGE_SORT=0"; do
    echo "== $e" >> $O/c128.txt
    env $e timeout -k 10 200 python3 tools/order_probe.py c128 $n 128 1.0 10 >> $O/c128.txt 2>> $O/c128.err || exit 1
  done
done
for e in "" "COSTA_TUNING=1 COSTA_LARGE_SORT=1"; do
  echo "== $e" >> $O/c128.txt
  env $e timeout -k 10 200 python3 tools/order_probe.py c128 16384 64 1.0 10 >> $O/c128.txt 2>> $O/c128.err || exit 1
done
