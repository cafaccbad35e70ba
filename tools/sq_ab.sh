#!/bin/bash
# large-shape ops of fp64 / c64 / c128 transposing lists on the square 64 x 64 sub-tile
# (COSTA_FORCE_SQ=1) against the list's own shape, 16384^2 'T', twice
set -o pipefail
O=gpurun_out/${1:-sq}; mkdir -p $O
for rep in 1 2; do
  for cfg in "c128 16384 128 1" "c128 16384 128 0" "f64 16384 256 0" "f64 16384 128 1" "c64 16384 128 0"; do
    for f in 0 1; do
      COSTA_FORCE_SQ=$f timeout -k 10 120 python3 tools/order_probe.py $cfg 10 2>/dev/null | sed "s/^/sq=$f /" >> $O/sq.txt || exit 1
    done
  done
done
