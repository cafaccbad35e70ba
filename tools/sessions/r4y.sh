#!/bin/bash
# r4 session y: transposes and copies at column strides off the powers of two (fp64 20480^2,
# 24576^2, 16384^2 at lld 49152): sub-tile orders, the fp64 128 x 64 / 128 x 128 shapes
set -o pipefail
O=gpurun_out/r4y
mkdir -p $O
timeout -k 10 120 tools/stride_probe segsizes > $O/segsizes.txt 2>&1 || exit 1
run() {  # label, env..., -- probe args
  local label=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done
  shift
  echo -n "$label " >> $O/matrix.txt
  env COSTA_TUNING=1 "${envs[@]}" timeout -k 10 200 python3 tools/order_probe.py "$@" >> $O/matrix.txt 2>> $O/err.txt
}
for g in "20480 0" "24576 0" "16384 32768"; do
  set -- $g
  n=$1; pad=$2
  run default COSTA_PROBE_LDPAD=$pad -- f64 $n 256 0.0 10 || exit 1
  run hint_order COSTA_PROBE_LDPAD=$pad COSTA_LARGE_SORT=1 -- f64 $n 256 0.0 10 || exit 1
  run f64w COSTA_PROBE_LDPAD=$pad COSTA_LIB=gpuvar/f64w/lib/libcosta_amd.so -- f64 $n 256 0.0 10 || exit 1
  run f64big COSTA_PROBE_LDPAD=$pad COSTA_LIB=gpuvar/f64big/lib/libcosta_amd.so -- f64 $n 256 0.0 10 || exit 1
  run f64big_hint COSTA_PROBE_LDPAD=$pad COSTA_LARGE_SORT=1 COSTA_LIB=gpuvar/f64big/lib/libcosta_amd.so -- f64 $n 256 0.0 10 || exit 1
  run copy_N COSTA_PROBE_LDPAD=$pad COSTA_PROBE_OP=N -- f64 $n 256 0.0 10 || exit 1
done
