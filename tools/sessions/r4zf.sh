#!/bin/bash
# r4 session zf: c128 square-class sub-tiles with longer source runs (128 x 64 with 512 / 1024
# threads, 128 x 32 with 256) against the shipped 64 x 64, destination order with panels
set -o pipefail
O=gpurun_out/r4zf
mkdir -p $O
for rep in 1 2; do
  for v in default c128w512 c128w1024 c128n; do
    lib=""
    [ $v != default ] && lib=gpuvar/$v/lib/libcosta_amd.so
    for a in "c128 32768 128 1.0 6" "c128 16384 128 1.0 10" "c128 16384 256 1.0 10"; do
      echo -n "$v " >> $O/shapes.txt
      COSTA_LIB=$lib timeout -k 10 200 python3 tools/order_probe.py $a >> $O/shapes.txt 2>> $O/err.txt || exit 1
    done
  done
done
