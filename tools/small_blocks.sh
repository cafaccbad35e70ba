#!/bin/bash
# 16384^2 'T' kernel rate with small and ragged blocks (the wavefront path), shipped library and
# the tuning builds under build/variants, beta = 0 and beta != 0
set -o pipefail
O=gpurun_out/${1:-smallblk}
mkdir -p $O
for lib in shipped build/variants/*/; do
  name=$(basename $lib)
  L=""; [ $lib != shipped ] && L=$lib/libcosta_amd.so
  for cfg in "f32 16384 16 0" "f32 16384 24 0" "f32 16384 28 0" "f32 16384 24 1" "f64 16384 16 0" "f64 16384 24 0" \
             "f64 16384 24 1" "c64 16384 24 0" "c128 16384 16 0" "c128 16384 24 1"; do
    COSTA_LIB=$L timeout -k 10 120 python3 tools/order_probe.py $cfg 10 2>/dev/null | sed "s/^/$name /" >> $O/small.txt || exit 1
  done
done
