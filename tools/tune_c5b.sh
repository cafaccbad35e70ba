#!/bin/bash
# cfg 5 'N': wavefront copy budget (COSTA_TINY_COPY_BUDGET bytes; larger ops are cut into pieces
# within it), interleaved, two repetitions.
#   usage (GPU box): tools/tune_c5b.sh > gpurun_out/c5b.log
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for rep in 1 2; do
    for b in 16384 8192 4096 2048 1024; do
        out=$(COSTA_TINY_COPY_BUDGET=$b timeout -k 10 120 python3 bench.py --workload cfg5 --cfg5-op N \
              --steps 10 --warmup 2 --no-cpu-baseline --no-e2e 2>/dev/null | grep '^{')
        rc=$?
        [ $rc -le 1 ] || { echo "stop rc=$rc"; exit $rc; }
        python3 -c "import json,sys; d=json.loads(sys.argv[1]); print('rep$rep budget=$b', d['value'], d['roofline']['achieved'])" "$out"
    done
done
