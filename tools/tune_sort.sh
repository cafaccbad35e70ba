#!/bin/bash
# cfg5: wavefront-path execution order (COSTA_TINY_SORT 3 hint / 2 dst / 1 src), repeated
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-sort}
mkdir -p "$OUT"
for rep in 1 2; do
  for op in N T; do
    for s in 3 2 1; do
      COSTA_TINY_SORT=$s timeout -k 10 300 python3 bench.py --workload cfg5 --cfg5-op $op --steps 20 \
          --warmup 3 --no-cpu-baseline --no-e2e > "$OUT/run.log" 2>&1 || { echo "failed $op $s"; tail -5 "$OUT/run.log"; exit 3; }
      python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], d['value'], d['kernel_node_GBps'])" \
          "$OUT/run.log" "rep$rep op=$op sort=$s" | tee -a "$OUT/sort.log"
    done
  done
done
