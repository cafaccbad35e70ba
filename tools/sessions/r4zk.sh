#!/bin/bash
# r4 session zk: fewer bytes in flight per CU for the fp64 transposes: one workgroup per CU
# (COSTA_TILE_LDS_MIN), 1024 threads per 64 x 128 sub-tile (4 loads per thread)
set -o pipefail
O=gpurun_out/r4zk
mkdir -p $O
for rep in 1 2; do
  for n in 16384 32768; do
    for v in "default" "lds81k:COSTA_TILE_LDS_MIN=83000" "t1024:COSTA_LIB=gpuvar/f64t1024/lib/libcosta_amd.so" "t1024_lds:COSTA_LIB=gpuvar/f64t1024/lib/libcosta_amd.so COSTA_TILE_LDS_MIN=83000"; do
      label=${v%%:*}; envs=""; [ "$label" != default ] && envs=${v#*:}
      echo -n "$label " >> $O/inflight.txt
      env COSTA_TUNING=1 $envs timeout -k 10 200 python3 tools/order_probe.py f64 $n 256 0.0 10 >> $O/inflight.txt 2>> $O/err.txt || exit 1
    done
  done
done
