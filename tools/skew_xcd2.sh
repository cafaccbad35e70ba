#!/bin/bash
# wide skew variant: parity of the unaligned tests, then the unaligned probe with the shipped
# grouping and with COSTA_SKEW_XCD = 0 / 4 / 16 (every skew list)
set -o pipefail
O=gpurun_out/${1:-skx2}
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_tiles.py -m gpu -k "unaligned or skew" > $O/pytest.log 2>&1 || exit 1
timeout -k 10 300 python3 tools/unaligned_probe.py 10 sides > $O/default.log 2>&1 || exit 1
for F in 0 4 16; do
  COSTA_SKEW_XCD=$F timeout -k 10 300 python3 tools/unaligned_probe.py 10 sides > $O/x$F.log 2>&1 || exit 1
done
timeout -k 10 300 python3 tools/unaligned_probe.py 10 sides > $O/default2.log 2>&1 || exit 1
