#!/bin/bash
# r4 session b: counters of cfg 5 'T' with the destination chunked / element-wise, and of cfg 4
set -o pipefail
O=gpurun_out/r4b
mkdir -p $O
tools/pmc_ab.sh $O/c5T 'chunk1:COSTA_TUNING=1 COSTA_TINY_CHUNK=1' 'chunk0:COSTA_TUNING=1 COSTA_TINY_CHUNK=0' -- --workload cfg5 --cfg5-op T --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-extra || exit 1
tools/pmc_ab.sh $O/c4 'def:COSTA_X=0' -- --workload cfg4 --edge 16384 --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-extra || exit 1
tools/pmc_ab.sh $O/c2 'def:COSTA_X=0' -- --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-extra || exit 1
