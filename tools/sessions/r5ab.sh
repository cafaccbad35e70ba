#!/bin/bash
# r5 session ab: the destination-block groups walked in XCD-contiguous slices (tuning build
# gpuvar/cbx, tile_kernels.hip COSTA_CB_XCD) against the shipped round-robin order: cfg 5 'T' /
# 'N' alternating, then one FETCH_SIZE pass of cfg 5 'T' each (L2 -> memory reads)
set -o pipefail
O=gpurun_out/r5ab
mkdir -p $O
export TMPDIR=/tmp
V=gpuvar
timeout -k 10 300 python3 tools/ab_bench.py $O/c5T 3 shipped: cbx:COSTA_LIB=$V/cbx/lib/libcosta_amd.so \
  -- --workload cfg5 --cfg5-op T --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --no-extra || exit 1
timeout -k 10 300 python3 tools/ab_bench.py $O/c5N 3 shipped: cbx:COSTA_LIB=$V/cbx/lib/libcosta_amd.so \
  -- --workload cfg5 --cfg5-op N --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --no-extra || exit 1
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_shipped -o p --output-format csv -- python3 bench.py --workload cfg5 --cfg5-op T --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-extra > $O/pmc_shipped.log 2>&1 || exit 1
python3 tools/pmc_brief.py $O/pmc_shipped 3221225472 > $O/pmc_shipped_summary.txt 2>&1
COSTA_LIB=$V/cbx/lib/libcosta_amd.so timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_cbx -o p --output-format csv -- python3 bench.py --workload cfg5 --cfg5-op T --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-extra > $O/pmc_cbx.log 2>&1 || exit 1
python3 tools/pmc_brief.py $O/pmc_cbx 3221225472 > $O/pmc_cbx_summary.txt 2>&1
