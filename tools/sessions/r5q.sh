#!/bin/bash
# r5 session q: destination-block groups with the flat element distribution (every load of a
# workgroup in flight at once; tile_kernels.hip COSTA_CB_FLAT) -- cblock / cfg 5 / tile tests,
# then cfg 5 'T' and 'N' against the per-op walk (gpuvar/cbold), alternating
set -o pipefail
O=gpurun_out/r5q
mkdir -p $O
PT="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 400 $PT tests/test_gpu_cblock.py tests/test_gpu_cfg5.py tests/test_gpu_tiles.py > $O/pytest.txt 2>&1 || exit 1
V=gpuvar
timeout -k 10 300 python3 tools/ab_bench.py $O/c5T 3 flat: old:COSTA_LIB=$V/cbold/lib/libcosta_amd.so \
  -- --workload cfg5 --cfg5-op T --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --no-extra || exit 1
timeout -k 10 300 python3 tools/ab_bench.py $O/c5N 3 flat: old:COSTA_LIB=$V/cbold/lib/libcosta_amd.so \
  -- --workload cfg5 --cfg5-op N --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --no-extra || exit 1
