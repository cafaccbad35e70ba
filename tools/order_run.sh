#!/bin/bash
# A/B of COSTA_LARGE_SORT (1 hint order, 2 destination-address order) across element types,
# block sizes and beta; every run its own process, two rounds:  tools/order_run.sh "CFG" ...
# with CFG = "DTYPE N BLOCK BETA" (tools/order_probe.py)
set -u
cd "${GRAFT_REPO_ROOT:-.}"
out=gpurun_out/order/order.log
mkdir -p gpurun_out/order
: > $out
for rep in 1 2; do
 for cfg in "$@"; do
  for s in 1 2; do
   COSTA_LARGE_SORT=$s timeout -k 10 120 python3 tools/order_probe.py $cfg 10 >> $out 2>/dev/null || { echo "fail $cfg $s" >> $out; exit 1; }
  done
 done
done
