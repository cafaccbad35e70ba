#!/bin/bash
# r4 session c: cfg 4 (c128 'T' alpha, beta, 32768^2) on other sub-tile shapes (the square
# variant's shape replaced in tuning builds, forced with COSTA_FORCE_SQ=1), and the host
# pipeline's time split for the end-to-end path
set -o pipefail
O=gpurun_out/r4c
mkdir -p $O
V=build/variants
sets=("def:")
for n in c1 c2 c3 c4 c5 c7; do sets+=("$n:COSTA_LIB=$V/$n/lib/libcosta_amd.so,COSTA_TUNING=1,COSTA_FORCE_SQ=1"); done
python3 tools/ab_bench.py $O/c4 1 "${sets[@]}" -- --workload cfg4 --edge 32768 --steps 5 --warmup 2 --no-cpu-baseline --no-e2e --no-extra || exit 1
COSTA_HOST_PIPE_TRACE=1 timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extra > $O/e2e.json 2> $O/e2e.err || exit 1
