#!/bin/bash
# skew sub-tile shapes (tuning builds under build/variants) on the unaligned probe, plus fp64
# sources read as misaligned 16-byte vectors
set -o pipefail
O=gpurun_out/${1:-skewshapes}
mkdir -p $O
timeout -k 10 300 python3 tools/unaligned_probe.py 10 sides > $O/shipped.log 2>&1 || exit 1
for v in build/variants/*/; do
  n=$(basename $v)
  COSTA_LIB=$v/libcosta_amd.so timeout -k 10 300 python3 tools/unaligned_probe.py 10 sides > $O/$n.log 2>&1 || exit 1
done
COSTA_MISALIGNED_VEC=2 timeout -k 10 300 python3 tools/unaligned_probe.py 10 sides > $O/misvec2.log 2>&1
