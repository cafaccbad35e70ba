#!/bin/bash
# cfg 5 'N' (a copy-only list): 1, 2 or 4 ops per wavefront moved together (COSTA_TINY_MULTI),
# interleaved, three repetitions.
#   usage (GPU box): tools/tune_c5m.sh > gpurun_out/c5m.log
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for rep in 1 2 3; do
    for m in 0 2 4; do
        out=$(COSTA_TINY_MULTI=$m timeout -k 10 120 python3 bench.py --workload cfg5 --cfg5-op N \
              --steps 10 --warmup 2 --no-cpu-baseline --no-e2e 2>/dev/null | grep '^{')
        rc=$?
        [ $rc -le 1 ] || { echo "stop rc=$rc"; exit $rc; }
        python3 -c "import json,sys; d=json.loads(sys.argv[1]); print('rep$rep multi=$m', d['value'], d['roofline']['achieved'])" "$out"
    done
done
