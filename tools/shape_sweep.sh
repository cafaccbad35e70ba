#!/bin/bash
# large-shape tuning builds (tools/tiny_variants.sh) x block sizes, 16384^2 'T':
#   tools/shape_sweep.sh "variant,variant" "CFG" "CFG" ...   (CFG as tools/order_probe.py)
set -u
cd "${GRAFT_REPO_ROOT:-.}"
out=gpurun_out/shapes/shapes.log
mkdir -p gpurun_out/shapes
: > $out
vars=$1
shift
for v in ${vars//,/ }; do
  for cfg in "$@"; do
   lib=""; [ $v != base ] && lib=build/variants/$v/libcosta_amd.so
   echo -n "$v: " >> $out
   COSTA_LIB=$lib timeout -k 10 120 python3 tools/order_probe.py $cfg 10 >> $out 2>/dev/null || { echo "fail $v $cfg" >> $out; exit 1; }
  done
done
