#!/bin/bash
# skew sub-tiles of fp64 lists grouped F s-neighbours per XCD (COSTA_SKEW_XCD_S), unaligned probe
set -o pipefail
O=gpurun_out/${1:-skews}; mkdir -p $O
for rep in 1 2; do
  for F in 0 2 4 8; do
    COSTA_SKEW_XCD_S=$F timeout -k 10 300 python3 tools/unaligned_probe.py 10 sides > $O/s${F}_$rep.log 2>&1 || exit 1
  done
done
