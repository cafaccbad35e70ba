#!/bin/bash
# r4 session r: copy lists (cfg 3 slice) in hint order (shipped), destination-address order, and
# destination order in 128 KiB panels
set -o pipefail
O=gpurun_out/r4r
mkdir -p $O
python3 tools/ab_bench.py $O/c3 2 'hint:' 'addr:COSTA_TUNING=1,COSTA_LARGE_SORT=2,COSTA_PANEL_ROWS=-1' 'panel:COSTA_TUNING=1,COSTA_LARGE_SORT=2' -- --workload cfg3 --steps 5 --warmup 2 --no-cpu-baseline --no-e2e --no-extra || exit 1
