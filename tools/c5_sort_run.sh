#!/bin/bash
# GPU box: tools/c5_sort_probe.py over the wavefront sort modes, local and loopback (pack/unpack)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-c5sort}
mkdir -p "$OUT"
for rep in 1 2; do
for lb in 0 1; do
  for op in N T; do
    for s in 4 5 2 3 1; do
      COSTA_LOOPBACK=$lb COSTA_TINY_SORT=$s timeout -k 10 120 python3 tools/c5_sort_probe.py $op 10 >> "$OUT/sort.log" 2>"$OUT/err.log"
      rc=$?
      [ $rc -eq 0 ] || { echo "rc=$rc lb=$lb op=$op s=$s"; tail "$OUT/err.log"; exit 1; }
    done
  done
done
done
cat "$OUT/sort.log"
