#!/bin/bash
# cfg 5 wavefront path: copy mode with 16-byte accesses (COSTA_TINY_VCOPY=1) against 4-byte
# element accesses (0), interleaved, three repetitions.
#   usage (GPU box): tools/tune_c5v.sh > gpurun_out/c5v.log
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for rep in 1 2 3; do
    for op in N T; do
        for v in 1 0; do
            out=$(COSTA_TINY_VCOPY=$v timeout -k 10 120 python3 bench.py --workload cfg5 --cfg5-op $op \
                  --steps 10 --warmup 2 --no-cpu-baseline --no-e2e 2>/dev/null | grep '^{')
            rc=$?
            [ $rc -le 1 ] || { echo "stop rc=$rc"; exit $rc; }
            python3 -c "import json,sys; d=json.loads(sys.argv[1]); print('rep$rep op=$op vcopy=$v', d['value'], d['roofline']['achieved'])" "$out"
        done
    done
done
