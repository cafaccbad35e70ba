#!/bin/bash
# -m gpu suite, then the unaligned probe with the shipped library and the tuning builds
set -o pipefail
O=gpurun_out/${1:-shift}; mkdir -p $O
[ -z "$NO_TESTS" ] && { timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 1; }
for rep in 1 2; do
  timeout -k 10 300 python3 tools/unaligned_probe.py 10 sides > $O/shipped_$rep.log 2>&1 || exit 1
  for v in build/variants/*/; do
    COSTA_LIB=$v/libcosta_amd.so timeout -k 10 300 python3 tools/unaligned_probe.py 10 sides > $O/$(basename $v)_$rep.log 2>&1 || exit 1
  done
done
