#!/bin/bash
# r4 session s: merging every op that continues another (large ones too) before sub-tiling,
# for block sizes that do not fill the sub-tiles (COSTA_MERGE=2)
set -o pipefail
O=gpurun_out/r4s
mkdir -p $O
for a in "c128 16384 80 1.0" "c128 16384 96 1.0" "f64 16384 96 0.0" "f64 16384 80 1.0" "c64 16384 80 0.0" "f32 16384 80 0.0" "f64 16384 256 0.0" "c128 16384 128 1.0" "f64 16384 100 0.0"; do
  for m in 1 2; do
    echo -n "merge=$m " >> $O/merge.txt
    COSTA_TUNING=1 COSTA_MERGE=$m timeout -k 10 200 python3 tools/order_probe.py $a 10 >> $O/merge.txt 2>> $O/merge.err || exit 1
  done
done
