#!/bin/bash
# GPU box (tuning, not product): fp64 16384^2 'T' with small blocks (tools/order_probe.py) for the
# default library and the fp64 transpose-shape variants under build/variants/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-small_block_ab}
mkdir -p "$OUT"
: > "$OUT/probe.log"
for rep in 1 2; do
for lib in default build/variants/*/; do
  n=$(basename "$lib")
  [ "$lib" = default ] && L="" || L="COSTA_LIB=${lib}libcosta_amd.so"
  for cfg in "f64 16384 64 0" "f64 16384 96 0" "f64 16384 64 1.5" "f64 16384 48 0"; do
    env $L timeout -k 10 120 python3 tools/order_probe.py $cfg 10 2>/dev/null | sed "s/^/$n /" >> "$OUT/probe.log"
    rc=${PIPESTATUS[0]}; [ $rc -eq 0 ] || { echo "rc=$rc $n $cfg"; exit 1; }
  done
done
done
sort -k3,3 -k5,5 -k1,1 "$OUT/probe.log"
