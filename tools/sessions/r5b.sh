#!/bin/bash
# r5 session b: destination-block groups (engine.cpp cblock_groups, tile_kernels.hip
# cblock_kernel) -- tile / cfg 5 tests, host pipelines with direct pack / unpack groups (and their
# per-case direct-group counts), the loopback exchange from page-locked memory; cfg 5 'T' / 'N'
# with the groups against the wavefront path (COSTA_CBLOCK=0), alternating
set -o pipefail
O=gpurun_out/r5b
mkdir -p $O
PT="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 400 $PT tests/test_gpu_cfg5.py tests/test_gpu_tiles.py > $O/pytest_tiles.txt 2>&1 || exit 1
COSTA_RECORD_HOST_DIRECT=$PWD/$O/host_direct.jsonl timeout -k 10 300 $PT tests/test_gpu_host_pipeline.py > $O/pytest_host.txt 2>&1 || exit 1
timeout -k 10 400 $PT tests/test_gpu_loopback.py > $O/pytest_loop.txt 2>&1 || exit 1
for op in T N; do
  timeout -k 10 300 python3 tools/ab_bench.py $O/c5$op 2 cblock: wave:COSTA_TUNING=1,COSTA_CBLOCK=0 \
    -- --workload cfg5 --cfg5-op $op --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --no-extra || exit 1
done
# the host pipeline's two-team mode (COSTA_HOST_TEAMS=1): host tests, then the end-to-end legs
COSTA_TUNING=1 COSTA_HOST_TEAMS=1 timeout -k 10 300 $PT tests/test_gpu_host_pipeline.py -k "not golden_host_pinned" > $O/pytest_host_teams.txt 2>&1 || exit 1
for r in 0 1; do
  for v in "one" "teams"; do
    if [ $v = teams ]; then E="COSTA_TUNING=1 COSTA_HOST_TEAMS=1"; else E=""; fi
    env $E COSTA_HOST_PIPE_TRACE=1 timeout -k 10 200 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-extra > $O/e2e_${v}_$r.json 2> $O/e2e_${v}_$r.err || exit 1
  done
done
