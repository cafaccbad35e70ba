#!/bin/bash
# unaligned destination: nt stores (0) / default-policy stores (1) / XCD slices (2) / both (3)
set -o pipefail
O=gpurun_out/${1:-unalmodes}
mkdir -p $O
for m in 0 1 2 3; do
  echo "== COSTA_MISDST_MODE=$m" >> $O/sides.log
  COSTA_MISDST_MODE=$m timeout -k 10 300 python3 tools/unaligned_probe.py 10 sides >> $O/sides.log 2>&1 || exit 1
done
echo "== COSTA_MISDST_MODE=3 COSTA_MISALIGNED_VEC=2" >> $O/sides.log
COSTA_MISDST_MODE=3 COSTA_MISALIGNED_VEC=2 timeout -k 10 300 python3 tools/unaligned_probe.py 10 sides >> $O/sides.log 2>&1
