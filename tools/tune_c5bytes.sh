#!/bin/bash
# A/B of the wavefront path's bytes in flight per lane (COSTA_TINY_BYTES: 64 default, 96, 128)
# on BASELINE cfg 5, both ops, interleaved twice.  Output: gpurun_out/<tag>/c5_bytes.log
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-c5bytes}
mkdir -p "$OUT"
for rep in 1 2; do
    for v in "N 64" "N 96" "N 128" "T 64" "T 96" "T 128"; do
        set -- $v
        COSTA_TINY_BYTES=$2 timeout -k 10 300 python3 bench.py --workload cfg5 --cfg5-op $1 \
            --steps 20 --warmup 3 --no-cpu-baseline --no-e2e > "$OUT/run.log" 2>&1 \
            || { echo "run failed: $v"; tail -5 "$OUT/run.log"; exit 3; }
        python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], d['value'], d['kernel_node_GBps'])" \
            "$OUT/run.log" "rep$rep op=$1 bytes=$2" | tee -a "$OUT/c5_bytes.log"
    done
done
