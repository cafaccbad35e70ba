#!/bin/bash
# r5 session z: c128's square sub-tile at 1024 threads (shipped now) -- the c128 / tile / parity
# tests, then cfg 4 at 16384^2 and 32768^2 against the r4 256-thread build (gpuvar/sq256)
set -o pipefail
O=gpurun_out/r5z
mkdir -p $O
PT="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 500 $PT tests/test_gpu_tiles.py tests/test_gpu_parity.py > $O/pytest.txt 2>&1 || exit 1
V=gpuvar
timeout -k 10 600 python3 tools/ab_bench.py $O/c4_16k 2 shipped: sq256:COSTA_LIB=$V/sq256/lib/libcosta_amd.so \
  -- --workload cfg4 --steps 10 --warmup 2 --no-cpu-baseline --no-e2e --no-extra || exit 1
timeout -k 10 700 python3 tools/ab_bench.py $O/c4_32k 2 shipped: sq256:COSTA_LIB=$V/sq256/lib/libcosta_amd.so \
  -- --workload cfg4 --edge 32768 --steps 5 --warmup 2 --no-cpu-baseline --no-e2e --no-extra || exit 1
