#!/bin/bash
# r5 session ag: destination-block groups ordered by their lowest source address (tuning
# COSTA_CBLOCK_ORDER=1) against destination order, cfg 5 'N' and 'T'
set -o pipefail
O=gpurun_out/r5ag
mkdir -p $O
L="shipped: src:COSTA_TUNING=1,COSTA_CBLOCK_ORDER=1"
timeout -k 10 300 python3 tools/ab_bench.py $O/c5N 3 $L \
  -- --workload cfg5 --cfg5-op N --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --no-extra || exit 1
timeout -k 10 300 python3 tools/ab_bench.py $O/c5T 3 $L \
  -- --workload cfg5 --cfg5-op T --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --no-extra || exit 1
