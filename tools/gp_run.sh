#!/bin/bash
# GPU box: tools/group_probe over its parameters, then the product's cfg 5 on the same lease
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-gp}
mkdir -p "$OUT"
: > "$OUT/probe.log"
for a in "T 4096 20 4 8 0" "T 4096 20 4 8 1" "T 4096 20 4 8 2" "N 4096 20 4 8 0" "N 4096 20 4 8 1" "N 4096 20 4 8 2" \
         "N 2048 20 4 8 1" "T 2048 20 4 8 1"; do
  timeout -k 10 120 tools/group_probe $a >> "$OUT/probe.log" 2>&1
  rc=$?
  [ $rc -eq 0 ] || { echo "rc=$rc $a"; cat "$OUT/probe.log"; exit 1; }
done
grep -E "kernel|WRONG" "$OUT/probe.log"
for s in 0 1 2 3; do
  COSTA_TINY_SORT=$s bash tools/ab_bench.sh "$OUT/ab" "c5N_sort$s|COSTA_TINY_SORT=$s|--workload cfg5 --cfg5-op N --steps 20 --warmup 3"
done
