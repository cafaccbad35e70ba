#!/bin/bash
# r5 session u: destination-block groups with chunked loads (tile_kernels.hip COSTA_CB_V2: the
# ops' 64-element chunks dealt round-robin to the wavefronts, up to 16 a wavefront in flight
# across op boundaries, descriptors requested with the header) -- cblock / cfg 5 / tile tests,
# then cfg 5 'T' and 'N' against the per-op walk (gpuvar/cbold), alternating
set -o pipefail
O=gpurun_out/r5u
mkdir -p $O
PT="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 400 $PT tests/test_gpu_cblock.py tests/test_gpu_cfg5.py tests/test_gpu_tiles.py > $O/pytest.txt 2>&1 || exit 1
V=gpuvar
timeout -k 10 300 python3 tools/ab_bench.py $O/c5T 3 v2: old:COSTA_LIB=$V/cbold/lib/libcosta_amd.so \
  -- --workload cfg5 --cfg5-op T --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --no-extra || exit 1
timeout -k 10 300 python3 tools/ab_bench.py $O/c5N 3 v2: old:COSTA_LIB=$V/cbold/lib/libcosta_amd.so \
  -- --workload cfg5 --cfg5-op N --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --no-extra || exit 1
