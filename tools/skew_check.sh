#!/bin/bash
# skew shape: parity of the unaligned tests, then the unaligned probe for the shipped build and
# every tuning build under build/variants
set -o pipefail
O=gpurun_out/${1:-skewcheck}
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
  -m gpu -k "unaligned" > $O/pytest.log 2>&1 || exit 1
bash tools/skew_shapes.sh ${1:-skewcheck}
