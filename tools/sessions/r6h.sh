#!/bin/bash
# r6 session h: destination-block groups -- chunk elements written to LDS in lane-rotated order
# (shipped now) against in order (gpuvar/norot); transposing groups on chunk loads with the
# rotation (gpuvar/vt); 8 KiB groups (gpuvar/c2); cfg 5 'N' and 'T'
set -o pipefail
O=gpurun_out/r6h
mkdir -p $O
export TMPDIR=/tmp
V=gpuvar
timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_cblock.py tests/test_gpu_cfg5.py > $O/pytest_rot.txt 2>&1 || exit 1
for v in vt c2; do
  COSTA_LIB=$V/$v/lib/libcosta_amd.so timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_cblock.py tests/test_gpu_cfg5.py > $O/pytest_$v.txt 2>&1 || exit 1
done
L="shipped: norot:COSTA_LIB=$V/norot/lib/libcosta_amd.so c2:COSTA_LIB=$V/c2/lib/libcosta_amd.so"
timeout -k 10 500 python3 tools/ab_bench.py $O/c5N 2 $L \
  -- --workload cfg5 --cfg5-op N --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --no-extra || exit 1
L="shipped: vt:COSTA_LIB=$V/vt/lib/libcosta_amd.so c2:COSTA_LIB=$V/c2/lib/libcosta_amd.so"
timeout -k 10 500 python3 tools/ab_bench.py $O/c5T 2 $L \
  -- --workload cfg5 --cfg5-op T --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --no-extra || exit 1
