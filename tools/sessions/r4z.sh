#!/bin/bash
# r4 session z: f-neighbour sub-tiles dispatched together in destination order (COSTA_PAIR_F)
set -o pipefail
O=gpurun_out/r4z
mkdir -p $O
for rep in 1 2; do
for g in "16384 0" "20480 0" "24576 0" "32768 0" "16384 32768"; do
  set -- $g
  for p in 0 2 4; do
    echo -n "pair $p " >> $O/pair.txt
    COSTA_TUNING=1 COSTA_PAIR_F=$p COSTA_PROBE_LDPAD=$2 timeout -k 10 200 python3 tools/order_probe.py f64 $1 256 0.0 10 >> $O/pair.txt 2>> $O/err.txt || exit 1
  done
done
done
for p in 0 2; do
  echo -n "pair $p " >> $O/pair.txt
  COSTA_TUNING=1 COSTA_PAIR_F=$p timeout -k 10 200 python3 tools/order_probe.py f32 20480 256 0.0 10 >> $O/pair.txt 2>> $O/err.txt || exit 1
  echo -n "pair $p " >> $O/pair.txt
  COSTA_TUNING=1 COSTA_PAIR_F=$p timeout -k 10 200 python3 tools/order_probe.py c64 20480 256 0.0 10 >> $O/pair.txt 2>> $O/err.txt || exit 1
done
