#!/bin/bash
# r6 session f: destination-block group variants on the r6 defaults (tuning builds: 16 chunks a lane
# in flight; 512 / 128 threads a group at the same 16 KiB budget), cfg 5 'N' and 'T'; the group
# builder's phases on the box (COSTA_PLAN_TRACE)
set -o pipefail
O=gpurun_out/r6f
mkdir -p $O
export TMPDIR=/tmp
V=gpuvar
for v in u16 t512 t128; do
  COSTA_LIB=$V/$v/lib/libcosta_amd.so timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_cblock.py tests/test_gpu_cfg5.py > $O/pytest_$v.txt 2>&1 || exit 1
done
L="shipped: u16:COSTA_LIB=$V/u16/lib/libcosta_amd.so t512:COSTA_LIB=$V/t512/lib/libcosta_amd.so t128:COSTA_LIB=$V/t128/lib/libcosta_amd.so"
timeout -k 10 700 python3 tools/ab_bench.py $O/c5N 2 $L \
  -- --workload cfg5 --cfg5-op N --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --no-extra || exit 1
L="shipped: t512:COSTA_LIB=$V/t512/lib/libcosta_amd.so t128:COSTA_LIB=$V/t128/lib/libcosta_amd.so"
timeout -k 10 500 python3 tools/ab_bench.py $O/c5T 2 $L \
  -- --workload cfg5 --cfg5-op T --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --no-extra || exit 1
for op in N T; do
  COSTA_PLAN_TRACE=1 timeout -k 10 300 python3 bench.py --workload cfg5 --cfg5-op $op --steps 5 --warmup 2 --no-cpu-baseline --no-e2e --no-extra > $O/trace_$op.json 2> $O/trace_$op.err || exit 1
done
