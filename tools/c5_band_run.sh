#!/bin/bash
# GPU box (tuning, not product): cfg 5 wavefront lists in the planner's hint order with the hint
# taken band-major (COSTA_HINT_BAND = rows per band; host planner) against destination order
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-c5band}
mkdir -p "$OUT"
: > "$OUT/band.log"
export COSTA_PLANNER=0
for rep in 1 2; do
  for op in N T; do
    for cfg in "5 0" "3 0" "3 256" "3 512" "3 1024" "3 2048" "3 4096"; do
      set -- $cfg
      COSTA_TINY_SORT=$1 COSTA_HINT_BAND=$2 timeout -k 10 120 python3 tools/c5_sort_probe.py $op 10 2>"$OUT/err.log" | sed "s/^/band=$2 /" >> "$OUT/band.log"
      rc=${PIPESTATUS[0]}
      [ $rc -eq 0 ] || { echo "rc=$rc $op $cfg"; tail "$OUT/err.log"; exit 1; }
    done
  done
done
cat "$OUT/band.log"
