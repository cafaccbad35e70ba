#!/bin/bash
# cfg5 sweep over the tiny-op kernel's knobs (COSTA_TINY_K, COSTA_TINY_CHUNKED); one line each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-tiny}
mkdir -p "$OUT"
for op in N T; do
  for ch in 0 1; do
    for k in ${KS:-1 2 4 8 16}; do
      COSTA_TINY_K=$k COSTA_TINY_CHUNKED=$ch timeout -k 10 300 python3 bench.py --workload cfg5 \
          --cfg5-op $op --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > "$OUT/$op.$ch.$k.log" 2>&1
      rc=$?
      if [ $rc -ne 0 ]; then echo "stop: $op $ch $k rc=$rc"; tail -5 "$OUT/$op.$ch.$k.log"; exit $rc; fi
      python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], d['value'], d['kernel_node_GBps'])" "$OUT/$op.$ch.$k.log" "$op chunked=$ch k=$k"
    done
  done
done
