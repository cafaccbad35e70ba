#!/bin/bash
# unaligned lld: element-wise guarded paths (shipped) against 16-byte accesses at 4-byte alignment
# on the destination (1), source (2) or both (3)
set -o pipefail
O=gpurun_out/${1:-unalmis}
mkdir -p $O
for m in 0 1 2 3; do
  echo "== COSTA_MISALIGNED_VEC=$m" >> $O/sides.log
  COSTA_TUNING=1 COSTA_MISALIGNED_VEC=$m timeout -k 10 300 python3 tools/unaligned_probe.py 10 sides >> $O/sides.log 2>&1 || exit 1
done
