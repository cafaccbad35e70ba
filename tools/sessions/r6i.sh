#!/bin/bash
# r6 session i: cfg 5 'N' copy groups' 16-byte chunk loads with the default cache policy
# (gpuvar/plain, COSTA_CB_NT 0) against non-temporal (shipped): tests, A/B, read bytes by size
set -o pipefail
O=gpurun_out/r6i
mkdir -p $O
export TMPDIR=/tmp
PL=gpuvar/plain/lib/libcosta_amd.so
COSTA_LIB=$PL timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_cblock.py tests/test_gpu_cfg5.py > $O/pytest_plain.txt 2>&1 || exit 1
timeout -k 10 500 python3 tools/ab_bench.py $O/c5N 3 "shipped:" "plain:COSTA_LIB=$PL" \
  -- --workload cfg5 --cfg5-op N --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --no-extra || exit 1
P="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_32B_sum"
COSTA_LIB=$PL timeout -s KILL 200 rocprofv3 --pmc $P -d $O/bytes_plain -o p --output-format csv -- python3 bench.py --workload cfg5 --cfg5-op N --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-extra > $O/bytes_plain.log 2>&1 || exit 1
python3 tools/pmc_bytes.py $O/bytes_plain 1073741824 > $O/bytes_plain.txt 2>&1
