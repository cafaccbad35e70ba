#!/bin/bash
# r4 session f: c128 'T' 128^2 blocks on 64 x 64 sub-tiles in destination order, the work list
# interleaved from K equal runs (K bands of target columns in flight at once)
set -o pipefail
O=gpurun_out/r4f
mkdir -p $O
for n in 32768 16384; do
  for k in 1 2 4 8 16 64; do
    echo "== K=$k" >> $O/c128.txt
    COSTA_TUNING=1 COSTA_FORCE_SQ=1 COSTA_LARGE_SORT=2 COSTA_LARGE_INTERLEAVE=$k timeout -k 10 200 python3 tools/order_probe.py c128 $n 128 1.0 10 >> $O/c128.txt 2>> $O/c128.err || exit 1
  done
done
for k in 1 2 4 8; do
  echo "== f64 K=$k" >> $O/c128.txt
  COSTA_TUNING=1 COSTA_LARGE_INTERLEAVE=$k timeout -k 10 200 python3 tools/order_probe.py f64 16384 256 0.0 10 >> $O/c128.txt 2>> $O/c128.err || exit 1
done
