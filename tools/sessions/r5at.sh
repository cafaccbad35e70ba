#!/bin/bash
# r5 session at: the destination-block store phase reading a lane's V image elements in rotated
# order (bank-conflict free; tuning build gpuvar/cbrot, COSTA_CB_ROT) -- the cblock tests on it,
# then cfg 5 'N' / 'T' against the shipped kernel
set -o pipefail
O=gpurun_out/r5at
mkdir -p $O
V=gpuvar
COSTA_LIB=$V/cbrot/lib/libcosta_amd.so timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_cblock.py tests/test_gpu_cfg5.py > $O/pytest.txt 2>&1 || exit 1
L="shipped: rot:COSTA_LIB=$V/cbrot/lib/libcosta_amd.so"
timeout -k 10 400 python3 tools/ab_bench.py $O/c5N 3 $L \
  -- --workload cfg5 --cfg5-op N --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --no-extra || exit 1
timeout -k 10 400 python3 tools/ab_bench.py $O/c5T 3 $L \
  -- --workload cfg5 --cfg5-op T --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --no-extra || exit 1
