#!/bin/bash
# r6 session j: the skew sub-tiles' 16-byte source loads with the default cache policy (gpuvar/
# skewdef) against non-temporal (shipped): tests, then tools/unaligned_probe.py sides, alternating
set -o pipefail
O=gpurun_out/r6j
mkdir -p $O
export TMPDIR=/tmp
SK=gpuvar/skewdef/lib/libcosta_amd.so
COSTA_LIB=$SK timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "unaligned_skew or unaligned_lld" > $O/pytest_skewdef.txt 2>&1 || exit 1
for r in 0 1; do
  timeout -k 10 300 python3 tools/unaligned_probe.py 10 sides > $O/shipped_$r.txt 2>&1 || exit 1
  COSTA_LIB=$SK timeout -k 10 300 python3 tools/unaligned_probe.py 10 sides > $O/skewdef_$r.txt 2>&1 || exit 1
done
