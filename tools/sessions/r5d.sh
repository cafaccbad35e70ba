#!/bin/bash
# r5 session d: host pipelines -- direct (DMA) pack / unpack groups from page-locked memory and
# their per-case direct-group counts (COSTA_RECORD_HOST_DIRECT), the loopback exchange from
# page-locked memory, the two-team mode (COSTA_HOST_TEAMS=1) against one pass per step on the
# end-to-end legs of the headline
set -o pipefail
O=gpurun_out/r5d
mkdir -p $O
PT="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
COSTA_RECORD_HOST_DIRECT=$PWD/$O/host_direct.jsonl timeout -k 10 300 $PT tests/test_gpu_host_pipeline.py > $O/pytest_host.txt 2>&1 || exit 1
timeout -k 10 400 $PT tests/test_gpu_loopback.py > $O/pytest_loop.txt 2>&1 || exit 1
COSTA_TUNING=1 COSTA_HOST_TEAMS=1 timeout -k 10 300 $PT tests/test_gpu_host_pipeline.py -k "not golden_host_pinned" > $O/pytest_host_teams.txt 2>&1 || exit 1
for r in 0 1; do
  for v in one teams; do
    if [ $v = teams ]; then E="COSTA_TUNING=1 COSTA_HOST_TEAMS=1"; else E="COSTA_TUNING=0"; fi
    env $E COSTA_HOST_PIPE_TRACE=1 timeout -k 10 200 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-extra > $O/e2e_${v}_$r.json 2> $O/e2e_${v}_$r.err || exit 1
  done
done
