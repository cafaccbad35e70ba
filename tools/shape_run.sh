#!/bin/bash
# fp32 large-shape variants (tools/tiny_variants.sh builds) on order_probe, two rounds
set -u
cd "${GRAFT_REPO_ROOT:-.}"
out=gpurun_out/shape/shape.log
mkdir -p gpurun_out/shape
: > $out
for rep in 1 2; do
 for v in base f128x256 f128x128 f256x64; do
  for cfg in "f32 16384 128 0" "f32 16384 256 0" "f32 16384 512 0" "f32 16384 128 2" "f32 16384 256 2"; do
   lib=""; [ $v != base ] && lib=build/variants/$v/libcosta_amd.so
   echo -n "$v: " >> $out
   COSTA_LIB=$lib timeout -k 10 120 python3 tools/order_probe.py $cfg 10 >> $out 2>/dev/null || { echo "fail $v $cfg" >> $out; exit 1; }
  done
 done
done
