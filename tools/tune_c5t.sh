#!/bin/bash
# cfg 5 'T': wavefront transpose budget (COSTA_TINY_LDS_BUDGET bytes of staged tile; larger ops
# are cut into near-square pieces within it), interleaved, two repetitions.
#   usage (GPU box): tools/tune_c5t.sh > gpurun_out/c5t.log
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for rep in 1 2; do
    for b in 8192 6144 4096 2048; do
        out=$(COSTA_TINY_LDS_BUDGET=$b timeout -k 10 120 python3 bench.py --workload cfg5 --cfg5-op T \
              --steps 10 --warmup 2 --no-cpu-baseline --no-e2e 2>/dev/null | grep '^{')
        rc=$?
        [ $rc -le 1 ] || { echo "stop rc=$rc"; exit $rc; }
        python3 -c "import json,sys; d=json.loads(sys.argv[1]); print('rep$rep lds_budget=$b', d['value'], d['roofline']['achieved'])" "$out"
    done
done
