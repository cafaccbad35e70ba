#!/bin/bash
# r4 session w: what the fp64 32768^2 transpose loses (4.0 against 6.2 TB/s at 16384^2):
# column stride against matrix size, segment size, other element types, copies
set -o pipefail
O=gpurun_out/r4w
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 tools/stride_probe strides > $O/stride_sweep.txt 2>&1 || exit 1
# fp64 16384^2 'T' at lld 16384 + pad (column strides 128 / 192 / 256 / 384 / 512 KiB)
for pad in 0 8192 16384 32768 49152; do
  COSTA_PROBE_LDPAD=$pad timeout -k 10 200 python3 tools/order_probe.py f64 16384 256 0.0 10 >> $O/f64_ld.txt 2>> $O/err.txt || exit 1
done
# sizes at ld = n
for n in 20480 24576 28672 32768; do
  timeout -k 10 200 python3 tools/order_probe.py f64 $n 256 0.0 10 >> $O/f64_n.txt 2>> $O/err.txt || exit 1
done
COSTA_PROBE_OP=N timeout -k 10 200 python3 tools/order_probe.py f64 32768 256 0.0 10 >> $O/f64_n.txt 2>> $O/err.txt || exit 1
# the square 64 x 64 shape at 32768^2
COSTA_TUNING=1 COSTA_FORCE_SQ=1 timeout -k 10 200 python3 tools/order_probe.py f64 32768 256 0.0 10 >> $O/f64_n.txt 2>> $O/err.txt || exit 1
# other element types at 256 KiB columns
for a in "f32 16384 256 0.0" "c64 16384 256 0.0" "c128 16384 128 0.0" "c64 32768 256 0.0"; do
  timeout -k 10 200 python3 tools/order_probe.py $a 10 >> $O/types.txt 2>> $O/err.txt || exit 1
done
COSTA_PROBE_LDPAD=16384 timeout -k 10 200 python3 tools/order_probe.py f32 16384 256 0.0 10 >> $O/types.txt 2>> $O/err.txt || exit 1
COSTA_PROBE_LDPAD=49152 timeout -k 10 200 python3 tools/order_probe.py f32 16384 256 0.0 10 >> $O/types.txt 2>> $O/err.txt || exit 1
# fp64 transposing shapes at 32768^2 and 16384^2: 128 x 64 (1 KiB read segments) and 128 x 128 / 1024 threads
for v in f64w f64big; do
  for n in 16384 32768; do
    echo -n "$v " >> $O/f64_shapes.txt
    COSTA_LIB=gpuvar/$v/lib/libcosta_amd.so timeout -k 10 200 python3 tools/order_probe.py f64 $n 256 0.0 10 >> $O/f64_shapes.txt 2>> $O/err.txt || exit 1
  done
done
