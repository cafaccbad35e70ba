#!/bin/bash
# r4 session zo: copy segment length against loads per thread; the fp64 64 x 64 transposing
# shape (forced) with 512 / 1024 threads (4 / 2 loads per thread)
set -o pipefail
O=gpurun_out/r4zo
mkdir -p $O
timeout -k 10 200 tools/stride_probe segu > $O/segu.txt 2>&1 || exit 1
for rep in 1 2; do
  for v in default sq512 sq1024; do
    envs="COSTA_TUNING=1"; [ $v != default ] && envs="COSTA_TUNING=1 COSTA_FORCE_SQ=1"
    [ $v = sq1024 ] && envs="$envs COSTA_LIB=gpuvar/sq1024/lib/libcosta_amd.so"
    echo -n "$v " >> $O/sq.txt
    env $envs timeout -k 10 200 python3 tools/order_probe.py f64 16384 256 0.0 20 >> $O/sq.txt 2>> $O/err.txt || exit 1
  done
done
