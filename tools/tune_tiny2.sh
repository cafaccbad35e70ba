#!/bin/bash
# cfg5: sort order x assignment x K for the tiny-op kernel (one bench line each)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-tiny2}
mkdir -p "$OUT"
run() {  # run <op> <sort> <chunked> <k>
  COSTA_TINY_SORT=$2 COSTA_TINY_CHUNKED=$3 COSTA_TINY_K=$4 timeout -k 10 300 python3 bench.py \
      --workload cfg5 --cfg5-op $1 --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > "$OUT/$1.$2.$3.$4.log" 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then echo "stop: $* rc=$rc"; tail -5 "$OUT/$1.$2.$3.$4.log"; exit $rc; fi
  python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], d['value'], d['kernel_node_GBps'])" "$OUT/$1.$2.$3.$4.log" "$1 sort=$2 chunked=$3 k=$4"
}
for op in N T; do
  for k in 2 4 8; do run $op 2 1 $k; done
  run $op 2 0 1
  run $op 1 1 4
done
