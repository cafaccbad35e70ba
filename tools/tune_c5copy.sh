#!/bin/bash
# A/B of the wavefront copy path's bytes per lane per pass (COSTA_TINY_COPY_BYTES 64 / 128) on
# BASELINE cfg 5, interleaved twice; 'T' once per setting.  Output: gpurun_out/<tag>/c5_copy.log
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-c5copy}
mkdir -p "$OUT"
for v in "N 64" "N 128" "N 64" "N 128" "T 64" "T 128"; do
    set -- $v
    COSTA_TINY_COPY_BYTES=$2 timeout -k 10 300 python3 bench.py --workload cfg5 --cfg5-op $1 \
        --steps 20 --warmup 3 --no-cpu-baseline --no-e2e > "$OUT/run.log" 2>&1 \
        || { echo "run failed: $v"; tail -5 "$OUT/run.log"; exit 3; }
    python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], d['value'], d['kernel_node_GBps'])" \
        "$OUT/run.log" "op=$1 copy_bytes=$2" | tee -a "$OUT/c5_copy.log"
done
