#!/bin/bash
# cfg5 kernel trace (per-launch times) and HBM PMC passes, plus a sort-order sweep.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-c5prof}
mkdir -p "$OUT"
export TMPDIR=/tmp COSTA_TINY_K=${COSTA_TINY_K:-1}
B="python3 bench.py --workload cfg5 --steps 5 --warmup 1 --no-cpu-baseline --no-e2e"
for op in N T; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/tr_$op" -o tr --output-format csv -- $B --cfg5-op $op > "$OUT/tr_$op.log" 2>&1 || exit $?
  for c in FETCH_SIZE WRITE_SIZE TCC_HIT_sum TCC_MISS_sum; do
    timeout -k 10 300 rocprofv3 --pmc $c -d "$OUT/pmc_${op}_$c" -o p --output-format csv -- $B --cfg5-op $op > "$OUT/pmc_${op}_$c.log" 2>&1 || exit $?
  done
done
for s in 0 1 2; do
  for op in N T; do
    COSTA_TINY_SORT=$s timeout -k 10 300 $B --cfg5-op $op > "$OUT/sort$s.$op.log" 2>&1 || exit $?
    python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], d['value'], d['kernel_node_GBps'])" "$OUT/sort$s.$op.log" "sort=$s $op"
  done
done
