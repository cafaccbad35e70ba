#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-.}"
out=gpurun_out/fo/fo.log
mkdir -p gpurun_out/fo
: > $out
for rep in 1 2; do
 for cfg in "f32 16384 128 0" "f32 16384 256 0" "f32 16384 512 0" "f32 16384 512 2"; do
  for v in "base 1" "base 2" "fold 1" "fold 2"; do
   set -- $v
   lib=""; [ $1 != base ] && lib=build/variants/$1/libcosta_amd.so
   echo -n "$1: " >> $out
   COSTA_LIB=$lib COSTA_LARGE_SORT=$2 timeout -k 10 120 python3 tools/order_probe.py $cfg 10 >> $out 2>/dev/null || { echo "fail" >> $out; exit 1; }
  done
 done
done
