#!/bin/bash
# cfg 5 wavefront path: ops per wavefront (COSTA_TINY_K) and their assignment (COSTA_TINY_CHUNKED:
# 0 = strided over the grid, 1 = contiguous chunks), interleaved, two repetitions.
#   usage (GPU box): tools/tune_c5k.sh > gpurun_out/c5k.log
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for rep in 1 2; do
    for op in N T; do
        for k in 1 2 4 8; do
            for ch in 0 1; do
                [ "$k" = 1 ] && [ "$ch" = 1 ] && continue
                out=$(COSTA_TINY_K=$k COSTA_TINY_CHUNKED=$ch timeout -k 10 120 python3 bench.py \
                      --workload cfg5 --cfg5-op $op --steps 10 --warmup 2 --no-cpu-baseline --no-e2e \
                      2>/dev/null | grep '^{')
                rc=$?
                [ $rc -le 1 ] || { echo "stop rc=$rc"; exit $rc; }
                python3 -c "import json,sys; d=json.loads(sys.argv[1]); print('rep$rep op=$op k=$k chunked=$ch', d['value'], d['roofline']['achieved'])" "$out"
            done
        done
    done
done
