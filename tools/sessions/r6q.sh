#!/bin/bash
# r6 session q: the small kernels of a list (skew sub-tiles, wavefront pieces) on a side stream
# overlapping the group / tile kernel (default) against one stream (COSTA_SIDE_STREAM=0): cfg 5
# 'N' / 'T' whole steps, alternating fresh processes; then the GPU tests that launch lists
set -o pipefail
O=gpurun_out/r6q
mkdir -p $O
export TMPDIR=/tmp
B="--steps 20 --warmup 3 --no-cpu-baseline --no-e2e --no-extra --workload cfg5"
timeout -k 10 600 python3 tools/ab_bench.py $O/N 3 "side:" "one:COSTA_TUNING=1,COSTA_SIDE_STREAM=0" -- $B --cfg5-op N > $O/N.log 2>&1 || exit 1
timeout -k 10 600 python3 tools/ab_bench.py $O/T 3 "side:" "one:COSTA_TUNING=1,COSTA_SIDE_STREAM=0" -- $B --cfg5-op T > $O/T.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_loopback.py tests/test_gpu_cfg5.py tests/test_gpu_cblock.py tests/test_gpu_parity.py > $O/pytest.txt 2>&1 || exit 1
