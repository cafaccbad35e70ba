#!/bin/bash
# r5 session b: destination-block groups (engine.cpp cblock_groups, tile_kernels.hip
# cblock_kernel) -- tile and cfg 5 tests; cfg 5 'T' / 'N' with the groups against the wavefront
# path (COSTA_CBLOCK=0) and tuning builds of the group kernel (elements in flight per lane,
# group budget, threads), alternating
set -o pipefail
O=gpurun_out/r5b
mkdir -p $O
PT="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 400 $PT tests/test_gpu_cfg5.py tests/test_gpu_tiles.py > $O/pytest_tiles.txt 2>&1 || exit 1
V=gpuvar
timeout -k 10 420 python3 tools/ab_bench.py $O/c5T 2 cblock: wave:COSTA_TUNING=1,COSTA_CBLOCK=0 \
  u8:COSTA_LIB=$V/cbU8/lib/libcosta_amd.so u32:COSTA_LIB=$V/cbU32/lib/libcosta_amd.so \
  c4:COSTA_LIB=$V/cbC4/lib/libcosta_amd.so t512:COSTA_LIB=$V/cbT512/lib/libcosta_amd.so \
  -- --workload cfg5 --cfg5-op T --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --no-extra || exit 1
timeout -k 10 200 python3 tools/ab_bench.py $O/c5N 2 cblock: wave:COSTA_TUNING=1,COSTA_CBLOCK=0 \
  -- --workload cfg5 --cfg5-op N --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --no-extra || exit 1
