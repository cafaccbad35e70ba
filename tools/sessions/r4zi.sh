#!/bin/bash
# r4 session zi: the loopback exchange tests with the alpha, beta 80^2-block multi-round case
set -o pipefail
O=gpurun_out/r4zi
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_loopback.py -x -v > $O/pytest.log 2>&1 || exit 1
