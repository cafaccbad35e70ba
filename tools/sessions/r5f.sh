#!/bin/bash
# r5 session f: destination-block groups at 16 KiB (default now; the r5e budget bug fixed: a range
# off the 16-byte grid needs V - 1 more elements of vectors) -- GPU tests, cfg 5 'T' / 'N' against
# the wavefront path; the headline's placement sensitivity (tools/offset_probe.py)
set -o pipefail
O=gpurun_out/r5f
mkdir -p $O
PT="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 400 $PT tests/test_gpu_cblock.py tests/test_gpu_cfg5.py tests/test_gpu_tiles.py > $O/pytest.txt 2>&1 || exit 1
timeout -k 10 300 python3 tools/ab_bench.py $O/c5T 2 cblock: wave:COSTA_TUNING=1,COSTA_CBLOCK=0 \
  -- --workload cfg5 --cfg5-op T --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --no-extra || exit 1
timeout -k 10 300 python3 tools/ab_bench.py $O/c5N 2 cblock: wave:COSTA_TUNING=1,COSTA_CBLOCK=0 \
  -- --workload cfg5 --cfg5-op N --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --no-extra || exit 1
timeout -k 10 300 python3 tools/offset_probe.py 2 > $O/offset.txt 2>&1 || exit 1
