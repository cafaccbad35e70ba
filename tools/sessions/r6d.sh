#!/bin/bash
# r6 session d: cfg 5 'N' destination-block groups with aligned 16-byte chunk loads (tuning builds:
# gpuvar/cbv, CB_UV 2 / 8 chunks a lane in flight, 32 KiB groups) in XCD column bands, against the
# shipped groups; the first call's host time with the rewritten group builder (COSTA_PLAN_TRACE)
set -o pipefail
O=gpurun_out/r6d
mkdir -p $O
export TMPDIR=/tmp
V=gpuvar
COSTA_LIB=$V/cbv/lib/libcosta_amd.so COSTA_TUNING=1 COSTA_CB_BANDS=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_cblock.py tests/test_gpu_cfg5.py > $O/pytest_cbv_bands.txt 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_cblock.py tests/test_gpu_cfg5.py > $O/pytest_shipped.txt 2>&1 || exit 1
B="COSTA_TUNING=1,COSTA_CB_BANDS=1"
L="shipped: cbv:COSTA_LIB=$V/cbv/lib/libcosta_amd.so,$B uv2:COSTA_LIB=$V/cbv_uv2/lib/libcosta_amd.so,$B uv8:COSTA_LIB=$V/cbv_uv8/lib/libcosta_amd.so,$B c8:COSTA_LIB=$V/cbv_c8/lib/libcosta_amd.so,$B"
timeout -k 10 700 python3 tools/ab_bench.py $O/c5N 2 $L \
  -- --workload cfg5 --cfg5-op N --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --no-extra || exit 1
for op in N T; do
  COSTA_PLAN_TRACE=1 timeout -k 10 300 python3 bench.py --workload cfg5 --cfg5-op $op --steps 5 --warmup 2 --no-cpu-baseline --no-e2e --no-extra > $O/trace_$op.json 2> $O/trace_$op.err || exit 1
done
