#!/bin/bash
# GPU box: tools/group_probe over its parameters, then the product's cfg 5 on the same lease
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-gp}
mkdir -p "$OUT"
: > "$OUT/probe.log"
for a in "T 4096 20 4 16" "T 8192 20 8 16" "T 4096 20 4 8" "T 2048 20 4 8" "T 8192 20 4 16" \
         "N 4096 20 4 16" "N 8192 20 8 16" "N 4096 20 4 8" "N 2048 20 4 8"; do
  timeout -k 10 120 tools/group_probe $a >> "$OUT/probe.log" 2>&1
  rc=$?
  [ $rc -eq 0 ] || { echo "rc=$rc $a"; cat "$OUT/probe.log"; exit 1; }
done
grep -E "kernel|WRONG" "$OUT/probe.log"
bash tools/ab_bench.sh "$OUT/ab" "c5N||--workload cfg5 --cfg5-op N --steps 20 --warmup 3" \
    "c5T||--workload cfg5 --cfg5-op T --steps 20 --warmup 3"
