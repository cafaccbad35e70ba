#!/bin/bash
# skew sub-tiles grouped by XCD (COSTA_SKEW_XCD=F) on the unaligned probe, shipped build and the
# tuning builds under build/variants
set -o pipefail
O=gpurun_out/${1:-skewxcd}
mkdir -p $O
for F in 0 2 4 8; do
  COSTA_SKEW_XCD=$F timeout -k 10 300 python3 tools/unaligned_probe.py 10 sides > $O/shipped_x$F.log 2>&1 || exit 1
  for v in build/variants/*/; do
    COSTA_LIB=$v/libcosta_amd.so COSTA_SKEW_XCD=$F timeout -k 10 300 python3 tools/unaligned_probe.py 10 sides > $O/$(basename $v)_x$F.log 2>&1 || exit 1
  done
done
