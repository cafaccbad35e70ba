#!/bin/bash
# r6 session o: 16-group XCD chunks and GPU-built lists through the engine -- the loopback
# exchange (unpack lists with GPU-built groups), the cfg 5 / group / work-list tests
set -o pipefail
O=gpurun_out/r6o
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_loopback.py > $O/pytest_lb.txt 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_work_lists.py tests/test_gpu_cblock.py tests/test_gpu_cfg5.py > $O/pytest_c5.txt 2>&1 || exit 1
